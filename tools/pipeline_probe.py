#!/usr/bin/env python3
"""Would two B-image forwards in flight at once (two contexts, two streams: consecutive batches pipelined) beat one
context's back-to-back forwards?  Most of a yolo11s x3 forward is one serial chain of kernels on one queue
(tools/trace_forward.py), each running alone on the GPU.  GPU only.

    python tools/pipeline_probe.py [--model s] [--batch 8] [--dtype x3] [--iters 100]
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
    ap.add_argument("--model", default="s")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="x3")
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    dev = torch.device("cuda", 0)
    B = a.batch
    for k in (1, 2, 3, 1, 2):
        models = [YOLO11Model(size=a.model, device="cuda:0", dtype=a.dtype, verbose=False) for _ in range(k)]
        xs = [synthetic_batch(B, 640, 1000 + i, dev) for i in range(k)]
        streams = [torch.cuda.Stream(dev) for _ in range(k)]
        for m, x, s in zip(models, xs, streams):
            with torch.cuda.stream(s):
                m.model.engine.run(x)
        torch.cuda.synchronize()

        def go(n):
            for i in range(n):
                j = i % k
                with torch.cuda.stream(streams[j]):
                    models[j].model.engine.run(xs[j])
        go(2 * k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        go(a.iters)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(f"{k} context(s) in flight: {dt * 1e3:.3f} ms per forward, {B / dt:.0f} img/s", flush=True)
        del models
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
