#!/usr/bin/env python3
"""Diagnostics for the LDS-DMA conv configs: per conv op, the relative error of its output buffer vs the same op run
with a first-generation kernel (cfg 0), for every DMA config pinned on that one op.  GPU only.

    python tools/dma_diag.py [--model n] [--batch 2] [--size 640]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

DMA_FIRST, NDMA = 17, 18


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=640)
    a = ap.parse_args()
    os.environ["YM_AUTOTUNE"] = "0"
    os.environ["YM_TUNE_TABLES"] = "0"
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(size=a.model, device="cuda:0", dtype="f16")
    eng = m.model.engine
    x = synthetic_batch(a.batch, a.size, 7, torch.device("cuda", 0))
    B, S = a.batch, a.size
    ops = eng.graph.ops
    eng.run(x, use_graph=False)
    convs = [i for i, op in enumerate(ops) if op.kind == "conv" and i > 1]
    bad = 0
    for cfg in range(DMA_FIRST, DMA_FIRST + NDMA):
        errs = []
        for i in convs:
            op = ops[i]
            d = op.args["dst"]
            dst = d.buf.id if hasattr(d, "buf") else d.id
            base = [-1] * len(ops)
            base[i] = 0
            eng.rt.set_op_cfg(B, S, S, base)
            eng.run(x, use_graph=False)
            ref = eng.read_buffer(dst, B).clone()
            base[i] = cfg
            eng.rt.set_op_cfg(B, S, S, base)
            eng.run(x, use_graph=False)
            got = eng.read_buffer(dst, B)
            rel = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
            errs.append((rel, op.name))
        worst = sorted(errs, reverse=True)[:4]
        nbad = sum(1 for r, _ in errs if r > 1e-2)
        bad += nbad
        print(f"cfg {cfg}: {nbad} ops > 1e-2; worst " + ", ".join(f"{n}={r:.3g}" for r, n in worst), flush=True)
    print("TOTAL BAD", bad)


if __name__ == "__main__":
    main()
