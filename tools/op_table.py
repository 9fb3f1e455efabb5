#!/usr/bin/env python3
"""Per-op table of one forward on the GPU: chosen conv config, replay device time (graph of back-to-back launches),
TFLOP/s, algorithmic GB/s and the roofline floor max(flops / MFMA peak, bytes / HBM peak).

    python tools/op_table.py [--model n] [--batch 8] [--size 640] [--dtype f16]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default="f16")
    a = ap.parse_args()
    from bench import PEAK_HBM_GBS, PEAK_TFLOPS, synthetic_batch
    from core.model import YOLO11Model
    blob = None
    if a.dtype == "i8":  # the PTQ plan of bench.py: calibration through the exact-f32 plan, qnnpack qconfig
        from yolomi.engine import Engine
        from yolomi.plan import pack_model
        from yolomi.quant import calibrate
        from yolomi.synth import synth_weights
        dev = torch.device("cuda", 0)
        ce = Engine(a.model, a.task, synth_weights(a.model, a.task, 0), dev, "f32")
        qp = calibrate(ce, [synthetic_batch(a.batch, a.size, 500 + i, dev) for i in range(4)], "qnnpack")
        del ce
        blob = pack_model(a.model, a.task, synth_weights(a.model, a.task, 0), "i8", qp)
    m = YOLO11Model(task=a.task, size=a.model, device="cuda:0", dtype=a.dtype, weights_blob=blob)
    eng = m.model.engine
    x = synthetic_batch(a.batch, a.size, 1000, torch.device("cuda", 0))
    eng.run(x)
    B, S = a.batch, a.size
    cfg = eng.rt.get_op_cfg(B, S, S) or [-1] * eng.rt.n_ops
    t = eng.profile_replay(x, reps=20)
    costs = eng.graph.op_costs(B, S, S, {"f16": 2, "f32": 4, "i8": 1, "f8": 1, "x3": 4}[a.dtype])
    tot = floor = 0.0
    print(f"yolo11{a.model} {a.task} B={B} {S}^2 {a.dtype}; tune source {eng.tune_source}")
    print(f"{'op':26s} {'kind':6s} {'shape':28s} {'cfg':>4s} {'us':>7s} {'floor':>6s} {'TF/s':>7s} {'GB/s':>7s}")
    for i, op in enumerate(eng.graph.ops):
        if t[i] < 0:
            continue
        fl, by = costs[i]
        us = t[i] * 1e3
        fl_us = max(fl / PEAK_TFLOPS[a.dtype] / 1e12, by / PEAK_HBM_GBS / 1e9) * 1e6
        tot += us
        floor += fl_us
        shape = ""
        if op.kind == "conv":
            ar = op.args
            s = ar["s"]
            M = B * (S // 8) ** 2  # placeholder, refined below
            H = S // (ar["dst"].buf.f if hasattr(ar["dst"], "buf") and ar["dst"].buf.f else 1)
            shape = f"k{ar['k']}s{s} N={ar['c2']} K={ar['k'] ** 2 * ar['c1']}"
        print(f"{op.name:26s} {op.kind:6s} {shape:28s} {cfg[i]:4d} {us:7.1f} {fl_us:6.1f} {fl / max(us, 1e-9) / 1e6:7.1f} "
              f"{by / max(us, 1e-9) / 1e3:7.0f}")
    print(f"total replay {tot:.1f} us, roofline floor {floor:.1f} us")


if __name__ == "__main__":
    main()
