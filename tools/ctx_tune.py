#!/usr/bin/env python3
"""In-context refinement of a conv tile table.  ym_tune times every candidate of an op in isolation (a graph of
back-to-back launches of that op alone: its input hot in L2); in the forward the input was just written by the
previous op on whichever XCDs ran it.  This tool takes the isolated top-K candidates of each conv op and keeps the one
that makes the WHOLE graph-replayed forward fastest (coordinate descent, A/B interleaved timing blocks), then writes
the refined table.  GPU only.

    python tools/ctx_tune.py [--model s] [--task detect] [--batch 8] [--top 3] [--out gpurun_out/ctx_table.json]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--block", type=int, default=40, help="forwards per timing block")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ctx_table.json"))
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    from yolomi.engine import TUNE_VERSION
    dev = torch.device("cuda", 0)
    m = YOLO11Model(task=a.task, size=a.model, device="cuda:0", dtype=a.dtype)
    eng = m.model.engine
    B, S = a.batch, a.size
    x = synthetic_batch(B, S, 1000, dev)
    eng.run(x)
    torch.cuda.synchronize()
    base = eng.rt.get_op_cfg(B, S, S)
    ops = eng.graph.ops
    # csrc/ym_conv.hip ids without the Bottleneck ones (17 first-gen + 30 DMA + 43 stream + 12 halo = 102, then 14
    # Bottleneck ids), plus the x3-only LDS-DMA ids appended after them in x3 plans
    nb0, nb1 = 102, 116
    nx = eng._ncfg() - (2 if a.dtype == "x3" else 0)  # x3: the last 2 ids are x3-only Bottleneck variants
    cands_all = [c for c in range(nx) if not nb0 <= c < nb1]
    print(f"source {eng.tune_source}, {len(cands_all)} conv configs", flush=True)
    # (ops on a fused Bottleneck id or a split pair keep it: the other families do not take a fused pair's shape;
    # a depthwise-fused 1x1 runs on csrc/ym_conv_dwpw.hip, whose ids are not these)
    conv = [i for i, op in enumerate(ops) if op.kind == "conv" and i > 1 and base[i] in cands_all
            and not op.args.get("dw")]

    # isolated per-op times of every config (graph of back-to-back launches per op, as ym_tune)
    iso = {}
    for c in cands_all:
        cfg = list(base)
        for i in conv:
            cfg[i] = c
        eng.rt.set_op_cfg(B, S, S, cfg)
        t = eng.profile_replay(x, reps=10)
        for i in conv:
            iso[(i, c)] = t[i]
    eng.rt.set_op_cfg(B, S, S, base)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def fwd_ms(cfg):
        eng.rt.set_op_cfg(B, S, S, cfg)
        eng.run(x)  # re-capture
        e0.record()
        for _ in range(a.block):
            eng.run(x)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / a.block

    def compare(c1, c2, rounds=3):
        t1, t2 = [], []
        for _ in range(rounds):
            t1.append(fwd_ms(c1))
            t2.append(fwd_ms(c2))
        return statistics.median(t1), statistics.median(t2)

    cur = list(base)
    t_base = statistics.median(fwd_ms(cur) for _ in range(5))
    print(f"base forward {t_base * 1e3:.1f} us", flush=True)
    changed = 0
    for i in sorted(conv, key=lambda i: -iso.get((i, base[i]), 0.0)):
        ranked = sorted((iso[(i, c)], c) for c in cands_all if iso[(i, c)] > 0)
        cands = []
        for _, c in ranked:
            if c != cur[i] and c not in cands:
                cands.append(c)
            if len(cands) >= a.top:
                break
        for c in cands:
            trial = list(cur)
            trial[i] = c
            t_cur, t_try = compare(cur, trial)
            if t_try < t_cur * 0.997:
                print(f"{ops[i].name:26s} {cur[i]:3d} -> {c:3d}: {t_cur * 1e3:.1f} -> {t_try * 1e3:.1f} us "
                      f"(isolated {iso[(i, cur[i])] * 1e3:.1f} vs {iso[(i, c)] * 1e3:.1f})", flush=True)
                cur = trial
                changed += 1
    t_new, t_old = compare(cur, base, rounds=5)
    print(f"refined {changed} ops: forward {t_old * 1e3:.1f} -> {t_new * 1e3:.1f} us", flush=True)
    if t_new < t_old:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump({"version": TUNE_VERSION, "device": torch.cuda.get_device_properties(dev).gcnArchName,
                   "ncfg": eng._ncfg(), "ops": [op.name for op in ops], "cfg": cur,
                   "note": f"tools/ctx_tune.py refinement of the isolated ym_tune table ({t_old * 1e3:.1f} -> "
                           f"{t_new * 1e3:.1f} us per graph-replayed forward)"}, open(a.out, "w"))
        print(f"wrote {a.out}")


if __name__ == "__main__":
    main()
