#!/usr/bin/env python3
"""Host-side cost of one predict() call, split: ctypes ym_infer (graph launch) enqueue time, device time, the
output clone + counts sync, Results construction.  GPU only.

    python tools/host_overhead.py [--model n] [--lanes 1]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--lanes", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    from core.results import Results
    m = YOLO11Model(size=a.model, device="cuda:0", dtype="f16")
    eng = m.model.engine
    eng.lanes = a.lanes
    x = synthetic_batch(8, 640, 1000, torch.device("cuda", 0))
    for _ in range(20):
        m.predict(x)
    torch.cuda.synchronize()
    t_enq = t_sync = t_res = t_tot = 0.0
    for _ in range(a.iters):
        t0 = time.perf_counter()
        dets, counts = eng.run(x)
        t1 = time.perf_counter()
        out = dets.clone()
        n = counts.tolist()
        t2 = time.perf_counter()
        _ = [Results.from_batch(x, b, m.model.names, out, n[b]) for b in range(8)]
        t3 = time.perf_counter()
        t_enq += t1 - t0
        t_sync += t2 - t1
        t_res += t3 - t2
        t_tot += t3 - t0
    k = 1e6 / a.iters
    print(f"lanes {a.lanes}: enqueue {t_enq * k:.1f} us, clone+sync {t_sync * k:.1f} us, Results {t_res * k:.1f} us, "
          f"total {t_tot * k:.1f} us per predict")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        m.predict(x)
    t1 = time.perf_counter()
    print(f"lanes {a.lanes}: predict() loop {(t1 - t0) * k:.1f} us per call")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        eng.run(x)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"lanes {a.lanes}: back-to-back enqueue {((t1 - t0) * k):.1f} us/launch, device {(t2 - t0) * k:.1f} us/forward")


if __name__ == "__main__":
    main()
