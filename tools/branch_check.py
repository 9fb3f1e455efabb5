#!/usr/bin/env python3
"""Does the branch schedule overlap on the GPU?  Forward time (device-bound loop of eng.run) for the branch
schedule and the serial order (YM_BRANCHES=1), eager launches and graph replays.  GPU only.

    python tools/branch_check.py [--model n] [--iters 100]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def bench(eng, x, use_graph, iters):
    for _ in range(5):
        eng.run(x, use_graph=use_graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        eng.run(x, use_graph=use_graph)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    x = synthetic_batch(8, 640, 1000, torch.device("cuda", 0))
    for br in ("4", "1"):  # branch schedule on 4 streams, serial
        os.environ["YM_BRANCHES"] = br
        m = YOLO11Model(size=a.model, device="cuda:0", dtype="f16", verbose=False)
        eng = m.model.engine
        print(f"branches={br}: eager {bench(eng, x, False, a.iters):.3f} ms  graph {bench(eng, x, True, a.iters):.3f} ms",
              flush=True)
        del m, eng
    del os.environ["YM_BRANCHES"]


if __name__ == "__main__":
    main()
