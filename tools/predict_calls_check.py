#!/usr/bin/env python3
"""Diagnostic: the detections of a fresh model's FIRST predict() call (graph capture), later calls and an eager
forward on the bench batch (yolo11s x3 B=8), compared row for row.

    python tools/predict_calls_check.py [s] [8]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from bench import synthetic_batch
    from core.model import YOLO11Model
    scale = sys.argv[1] if len(sys.argv) > 1 else "s"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    x = synthetic_batch(B, 640, 1000, dev)
    m = YOLO11Model(task="detect", size=scale, device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    calls = {}
    for name, kw in (("first", {}), ("second", {}), ("third_sync", {"sync": True})):
        res = m.predict(x, **kw)
        calls[name] = [r.boxes.data.clone() for r in res]
    rows, counts = eng.run(x, use_graph=False)
    torch.cuda.synchronize()
    n = counts.tolist()
    calls["eager"] = [rows[b, :n[b], :6].clone() for b in range(B)]
    rows, counts = eng.run(x)  # graph, engine-owned rows
    torch.cuda.synchronize()
    n = counts.tolist()
    calls["graph_engine_rows"] = [rows[b, :n[b], :6].clone() for b in range(B)]
    ref = calls["eager"]
    for name, got in calls.items():
        same = all(a.shape == b.shape and torch.equal(a, b) for a, b in zip(got, ref))
        diffs = [float((a - b).abs().max()) if a.shape == b.shape and a.numel() else (-1.0 if a.shape != b.shape else 0.0)
                 for a, b in zip(got, ref)]
        print(f"{name:18s} counts {[len(g) for g in got]} bitwise-equal-to-eager {same} max|diff| per image {diffs}",
              flush=True)


if __name__ == "__main__":
    main()
