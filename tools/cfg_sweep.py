#!/usr/bin/env python3
"""Per-op x per-config replay times (µs) for one workload: pins config c on every conv (inapplicable ops fall back to
the heuristic, shown as '-') and times each op as a graph of back-to-back launches.  GPU only.

    python tools/cfg_sweep.py [--model s] [--batch 8] [--size 640] [--ops regex]
"""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--ops", default=".")
    ap.add_argument("--cfgs", default="0-40")
    a = ap.parse_args()
    os.environ["YM_AUTOTUNE"] = "0"
    os.environ["YM_TUNE_TABLES"] = "0"
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(size=a.model, device="cuda:0", dtype="f16")
    eng = m.model.engine
    x = synthetic_batch(a.batch, a.size, 1000, torch.device("cuda", 0))
    B, S = a.batch, a.size
    eng.run(x)
    cfgs = []
    for part in a.cfgs.split(","):
        lo, _, hi = part.partition("-")
        cfgs += list(range(int(lo), int(hi or lo) + 1))
    ops = eng.graph.ops
    sel = [i for i, op in enumerate(ops) if op.kind == "conv" and i > 1 and re.search(a.ops, op.name)]
    tab = {}
    for c in cfgs:
        eng.rt.set_op_cfg(B, S, S, [c if op.kind == "conv" else -1 for op in ops])
        t = eng.profile_replay(x, reps=20)
        for i in sel:
            tab[(i, c)] = t[i] * 1e3
        print(f"cfg {c} done", file=sys.stderr, flush=True)
    print(f"{'op':24s} " + " ".join(f"{c:>5d}" for c in cfgs) + "   best")
    for i in sel:
        row = [tab[(i, c)] for c in cfgs]
        b = min(range(len(cfgs)), key=lambda k: row[k])
        print(f"{ops[i].name:24s} " + " ".join(f"{v:5.1f}" for v in row) + f"   {cfgs[b]}:{row[b]:.1f}")


if __name__ == "__main__":
    main()
