#!/usr/bin/env python3
"""Headline benchmark: images/s of batched YOLO11 inference at 640x640 on MI355X (+ mAP50-95 vs the CPU oracle).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model n] [--batch 8] [--size 640] [--dtype f16]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one `YOLO11Model.predict(batch)` call (the reference's timed unit: core/model.py:277-282,
benchmarks/speed_benchmark.py:330-335) over B=8 synthetic U[0,1) 640x640 images already resident in HBM:
input /255 rule → yolo11n forward (one HIP-graph replay) → decode → NMS → per-image Results (one D2H sync).
Multi-GPU: one process per GPU, rank 0 packs the weights once and broadcasts the blob over RCCL (xGMI); each rank
then runs its own batch shard with no per-step collective ("weak" scaling: 8 images per GPU per step).

Rank 0 prints ONE JSON line.  Extra fields: `roofline` (conv implicit-GEMM kernels, live HIP-event timing),
`cpu_baseline` (the oracle on host cores, N=1 only), `accuracy` (mAP50-95 of GPU detections against oracle
detections as pseudo ground truth, N=1 only), `device_images_per_s` (back-to-back graph replays, no host sync).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec @640×640 (1/2/4/8 MI355X) + mAP50-95 vs CPU ref"
PEAK_TFLOPS = {"f16": 2500.0, "f32": 157.3, "i8": 5000.0}  # dense MFMA peaks (MI355X_MICROARCH.md; i8 = TOP/s)
ACT_BYTES = {"f16": 2, "f32": 4, "i8": 1}
PEAK_HBM_GBS = 8000.0


def synthetic_batch(B, S, seed, device):
    from yolomi.synth import uniform
    x = uniform(seed, B * 3 * S * S).astype(np.float32).reshape(B, 3, S, S)
    return torch.from_numpy(x).to(device)


def pmc_traffic(workload):
    """HBM-side bytes per forward of the conv family from the newest committed PMC summary of this workload
    (profiles/<round>_pmc.json, produced by tools/rocprof_summary.py from separate rocprofv3 --pmc passes)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json"))):
        try:
            j = json.load(open(p))
        except (OSError, ValueError):
            continue
        # the summary names the network/batch/dtype; the bench line appends how it was driven (", predict() loop")
        if j.get("workload") == workload.split(",")[0] and "conv" in j.get("families", {}):
            best = (p, j)
    if best is None:
        return None, None
    return best[1]["families"]["conv"]["bytes_corrected"], os.path.relpath(best[0], ROOT)


def conv_roofline(model, x, dtype, workload, reps=20):
    """Live per-op device times on the launch stream → conv-family roofline.

    Each conv launch of the forward is captured as a HIP graph of `reps` back-to-back launches on the real
    activation buffers and bracketed by one HIP event pair (ym_profile_replay): per-launch device time without the
    per-op marker packets an eager event pair would add.  `achieved` = Σ algorithmic FLOPs of the forward's conv
    launches ÷ Σ their per-launch times (per-unit figures: DESIGN.md §4)."""
    eng = model.model.engine
    B, _, H, W = x.shape
    Bl = eng.lane_batch(B)  # every kernel of a lane sees Bl images: time and count one lane's launches
    x = x[:Bl]
    costs = eng.graph.op_costs(Bl, H, W, ACT_BYTES[dtype])
    times = np.array(eng.profile_replay(x, reps=reps))
    eng.run(x, lanes=1)  # restore the buffers the replay clobbered
    kinds = [op.kind for op in eng.graph.ops]
    conv = [i for i, k in enumerate(kinds) if k == "conv"]
    t_conv = float(times[conv].sum()) * 1e-3
    fl = float(sum(costs[i][0] for i in conv))
    by = float(sum(costs[i][1] for i in conv))
    per_kind = {}
    for k, t in zip(kinds, times):
        if t >= 0:
            per_kind[k] = per_kind.get(k, 0.0) + float(t)
    top = sorted(((float(times[i]), eng.graph.ops[i].name, costs[i][0] / max(times[i] * 1e-3, 1e-12) / 1e12)
                  for i in conv), reverse=True)[:8]
    ach = fl / t_conv / 1e12
    traffic, tsrc = pmc_traffic(workload)
    return {
        "bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_TFLOPS[dtype], "unit": "TFLOP/s",
        "frac": round(ach / PEAK_TFLOPS[dtype], 4), "traffic": traffic,
        "traffic_note": (f"HBM-side bytes per forward of all conv launches (PMC FETCH_SIZE x2 + WRITE_SIZE, {tsrc}); "
                         f"algorithmic bytes per forward {int(by)}") if traffic else "no PMC summary for this workload",
        "kernel": "conv implicit GEMM (%s): all %d conv launches of one lane's forward (%d images), aggregated%s"
                  % ("conv_i8, v_mfma_i32_32x32x32_i8" if dtype == "i8" else "conv_igemm/conv_lds/conv_dma", len(conv),
                     Bl, "; int8 ops counted as FLOPs" if dtype == "i8" else ""),
        "timing": f"HIP events around a graph of {reps} back-to-back launches per op, on the launch stream",
        "launches": len(conv), "avg_launch_us": round(t_conv / len(conv) * 1e6, 2),
        "flops_per_forward": fl, "bytes_per_forward_algorithmic": by,
        "hbm_algorithmic_GBps": round(by / t_conv / 1e9, 1), "hbm_frac": round(by / t_conv / 1e9 / PEAK_HBM_GBS, 4),
        "ms_by_kind_replay": {k: round(v, 4) for k, v in per_kind.items()},
        "top_convs": [{"op": n, "ms": round(t, 4), "tflops": round(tf, 1)} for t, n, tf in top],
    }


def cpu_baseline(scale, task, x_gpu_dets, xs, seconds, qparams=None):
    """Oracle (torch CPU fp32, fused; or the int8 oracle of oracle/quant.py for an int8 run) timed on this host; also
    mAP of the GPU dets against the oracle's dets (and, for int8, against the float oracle's: the quantisation loss)."""
    from oracle.predict import OracleModel
    from yolomi.metrics import evaluate
    from yolomi.synth import synth_weights
    nthreads = int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))
    torch.set_num_threads(nthreads)
    if qparams is not None:
        from oracle.quant import Int8OracleModel
        om = Int8OracleModel(scale, task, synth_weights(scale, task, 0), qparams)
    else:
        om = OracleModel(scale, task, synth_weights(scale, task, 0))
    x1 = xs[:1].cpu()
    om.predict(x1)  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        om.predict(x1)
        n += 1
    dt = time.perf_counter() - t0
    ref = om.predict(xs.cpu())
    gts = [r["boxes"].numpy() for r in ref]
    m = evaluate(x_gpu_dets, gts)
    try:
        cpu_name = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")),
                        "unknown")
    except OSError:
        cpu_name = "unknown"
    what = "int8 oracle (oracle/quant.py: integer convs as exact float64 convs)" if qparams else "oracle"
    base = {"value": round(n / dt, 3), "unit": "images/s", "cores": nthreads, "kind": "port",
            "sample": f"{what} predict yolo11{scale} B=1 640x640 U[0,1): {n} images in {dt:.1f}s on {cpu_name} "
                      f"(os.cpu_count={os.cpu_count()})"}
    acc = {"map50_95": round(m["map"], 4), "map50": round(m["map50"], 4), "images": len(gts),
           "gt": ("int8 oracle (CPU) detections, same qparams, as pseudo ground truth" if qparams else
                  "oracle (CPU fp32) detections as pseudo ground truth"),
           "dets_gpu": int(sum(len(d) for d in x_gpu_dets)), "dets_oracle": int(sum(len(g) for g in gts))}
    if qparams is not None:  # quantisation loss: int8 GPU detections vs the float oracle's
        fl = OracleModel(scale, task, synth_weights(scale, task, 0)).predict(xs.cpu())
        mf = evaluate(x_gpu_dets, [r["boxes"].numpy() for r in fl])
        acc["vs_fp32_oracle"] = {"map50_95": round(mf["map"], 4), "map50": round(mf["map50"], 4)}
    return base, acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="n")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--batch", type=int, default=8, help="images per GPU per step")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default="f16", choices=["f16", "f32", "i8"])
    ap.add_argument("--backend", default="qnnpack", choices=["qnnpack", "fbgemm"], help="i8: PTQ qconfig")
    ap.add_argument("--calib-batches", type=int, default=4, help="i8: calibration batches (B images each)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--lanes", type=int, default=int(os.environ.get("YM_LANES", "1")),
                    help="concurrent image slices per forward graph (yolomi lanes)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from core.model import YOLO11Model
    from yolomi.plan import pack_model
    from yolomi.synth import synth_weights

    # weights: packed once on rank 0, broadcast over RCCL as one uint8 blob.  i8: rank 0 first runs the PTQ
    # calibration (exact-f32 plan + torch.ao observers, yolomi.quant) on synthetic batches disjoint from the timed one
    t_init = time.perf_counter()
    qp = None
    if rank == 0 and a.dtype == "i8":
        from yolomi.engine import Engine
        from yolomi.quant import calibrate
        ce = Engine(a.model, a.task, synth_weights(a.model, a.task, 0), dev, "f32")
        qp = calibrate(ce, [synthetic_batch(a.batch, a.size, 500 + i, dev) for i in range(a.calib_batches)],
                       a.backend)
        del ce
    if rank == 0:
        blob = pack_model(a.model, a.task, synth_weights(a.model, a.task, 0), a.dtype, qp)
        nbytes = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    else:
        blob, nbytes = None, torch.zeros(1, dtype=torch.int64, device=dev)
    if world > 1:
        dist.broadcast(nbytes, 0)
        buf = (torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev) if rank == 0
               else torch.empty(int(nbytes.item()), dtype=torch.uint8, device=dev))
        dist.broadcast(buf, 0)
        blob = bytes(buf.cpu().numpy())
    model = YOLO11Model(task=a.task, size=a.model, device=f"cuda:{local}", dtype=a.dtype, weights_blob=blob)
    model.model.engine.lanes = a.lanes
    init_s = time.perf_counter() - t_init

    B = a.batch
    x = synthetic_batch(B, a.size, 1000 + rank, dev)
    for _ in range(a.warmup):
        model.predict(x)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = model.predict(x)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    value = world * B * a.steps / elapsed

    # device-side throughput: back-to-back graph replays without the per-batch host sync of predict()
    eng = model.model.engine
    for _ in range(5):
        eng.run(x)
    torch.cuda.synchronize()
    td = time.perf_counter()
    for _ in range(a.steps):
        eng.run(x)
    torch.cuda.synchronize()
    dev_ips = B * a.steps / (time.perf_counter() - td)

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.dtype, "data": "synthetic",
        "config": {"workload": f"yolo11{a.model} {a.task} {a.size}x{a.size} batch {B}/GPU {a.dtype}, predict() loop",
                   "batch_per_gpu": B, "global_batch": B * world, "image_size": a.size,
                   "parallelism": f"dp{world} (batch-sharded, RCCL weight broadcast)"},
        "device_images_per_s": round(dev_ips * world, 2),
        "init_s": round(init_s, 3),
    }
    Bl = model.model.engine.lane_batch(B)
    out["config"]["lanes"] = -(-B // Bl)
    out["config"]["conv_tiles"] = model.model.engine.tune_source.get((Bl, a.size, a.size), "heuristic")
    if rank == 0 and not a.no_roofline:
        out["roofline"] = conv_roofline(model, x, a.dtype, out["config"]["workload"])
    if rank == 0 and world == 1 and not a.no_cpu:
        gdets = [r.boxes.data.cpu().numpy() for r in res]
        base, acc = cpu_baseline(a.model, a.task, gdets, x, a.cpu_seconds, qp)
        out["cpu_baseline"] = base
        out["accuracy"] = acc
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
