#!/usr/bin/env python3
"""Eager forwards of the bench workload for rocprofv3 PMC passes (one counter group per run, no trace domains).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 tools/pmc_forward.py

Uses the same tuned conv tables as bench.py (YM_TUNE_DIR / yolomi/tuned), so the dispatch sequence of the last
`--reps` forwards is exactly one bench forward each; tools/rocprof_summary.py splits them at the input_stats kernel.
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ops-out", default=None, help="write the op names of one forward, in launch order, to this file")
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    blob = None
    if a.dtype in ("i8", "f8"):  # the PTQ plan of bench.py: calibration through the exact-f32 plan
        from yolomi.engine import Engine
        from yolomi.plan import pack_model
        from yolomi.quant import calibrate
        from yolomi.synth import synth_weights
        d0 = torch.device("cuda", 0)
        ce = Engine(a.model, a.task, synth_weights(a.model, a.task, 0), d0, "f32")
        qp = calibrate(ce, [synthetic_batch(a.batch, a.size, 500 + i, d0) for i in range(4)],
                       "fp8" if a.dtype == "f8" else "qnnpack")
        del ce
        blob = pack_model(a.model, a.task, synth_weights(a.model, a.task, 0), a.dtype, qp)
    m = YOLO11Model(task=a.task, size=a.model, device="cuda:0", dtype=a.dtype, weights_blob=blob)
    x = synthetic_batch(a.batch, a.size, 1000, torch.device("cuda", 0))
    eng = m.model.engine
    eng.run(x, use_graph=False)  # table lookup (or tuning) happens here
    torch.cuda.synchronize()
    if a.ops_out:
        # name, kind, kernel launches of the op (a split pair launches two), algorithmic FLOPs and bytes
        cfg = eng.rt.get_op_cfg(a.batch, a.size, a.size) or [0] * len(eng.graph.ops)
        costs = eng.graph.op_costs(a.batch, a.size, a.size, {"i8": 1, "f8": 1, "f32": 4, "x3": 4}.get(a.dtype, 2))
        with open(a.ops_out, "w") as f:
            for op, c, (fl, by) in zip(eng.graph.ops, cfg, costs):
                # (the input op is one input_stats launch since round 6's per-step /255 rule: counting it as two
                # shifted every later row of the per-op table by one dispatch)
                n = 2 if op.kind == "conv" and c >= (1 << 20) else 1
                f.write(f"{op.name}\t{op.kind}\t{n}\t{int(fl)}\t{int(by)}\n")
    for _ in range(a.reps):
        eng.run(x, use_graph=False)
    torch.cuda.synchronize()
    print(f"pmc_forward: {a.reps} eager forwards of yolo11{a.model} B={a.batch} {a.size}^2 {a.dtype}; tune source "
          f"{eng.tune_source}")


if __name__ == "__main__":
    main()
