#!/usr/bin/env python3
"""Does splitting one B-image forward into two concurrent half-batch forwards on two HIP streams (two contexts, two
graphs, two hardware queues) beat the single B-image graph?  The 20x20 / 40x40 layers of a B = 8 forward fill only
100-400 workgroups, so two independent forwards could share the idle CUs.  GPU only.

    python tools/concur_probe.py [--model s] [--batch 8] [--iters 200]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--splits", default="2,4")
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    dev = torch.device("cuda", 0)
    B = a.batch
    x = synthetic_batch(B, 640, 1000, dev)
    m = YOLO11Model(size=a.model, device="cuda:0", dtype="f16")
    e = m.model.engine
    t_one = timed(lambda: e.run(x), a.iters)
    print(f"one context, B={B} graph: {t_one:.3f} ms/forward ({B / t_one * 1e3:.0f} img/s)", flush=True)
    for k in [int(s) for s in a.splits.split(",")]:
        Bk = B // k
        models = [YOLO11Model(size=a.model, device="cuda:0", dtype="f16") for _ in range(k)]
        engs = [mm.model.engine for mm in models]
        xs = [x[i * Bk:(i + 1) * Bk].contiguous() for i in range(k)]
        streams = [torch.cuda.Stream(dev) for _ in range(k)]
        for eg, xi in zip(engs, xs):  # tune / capture outside the timed region
            eg.run(xi)
        torch.cuda.synchronize()

        def seq():
            for eg, xi in zip(engs, xs):
                eg.run(xi)

        def conc():
            cur = torch.cuda.current_stream(dev)
            for s in streams:
                s.wait_stream(cur)
            for eg, xi, s in zip(engs, xs, streams):
                with torch.cuda.stream(s):
                    eg.run(xi)
            for s in streams:
                cur.wait_stream(s)

        t_seq = timed(seq, a.iters)
        t_conc = timed(conc, a.iters)
        print(f"{k} contexts x B={Bk}: sequential {t_seq:.3f} ms, concurrent streams {t_conc:.3f} ms "
              f"({B / t_conc * 1e3:.0f} img/s, {t_one / t_conc:.2f}x the single graph)", flush=True)


if __name__ == "__main__":
    main()
