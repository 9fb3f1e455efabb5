#!/usr/bin/env python3
"""Where the segment predict() loop spends its time beyond the device forward (yolo11s-seg B=4 640²): wall per
step of (a) graph replay + counts sync, (b) + dets clone, (c) + mask kernels + non-empty sync, (d) full predict()."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(task="segment", size=sys.argv[1] if len(sys.argv) > 1 else "s", device="cuda:0")
    eng = m.model.engine
    x = synthetic_batch(4, 640, 1000, torch.device("cuda", 0))
    for _ in range(10):
        m.predict(x)
    torch.cuda.synchronize()

    def t(fn, n=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    def a():
        d, c = eng.run(x)
        return c.tolist()

    def b():
        d, c = eng.run(x)
        o = d[:4].clone()
        return c[:4].tolist()

    def c():
        d, cc = eng.run(x)
        o = d[:4].clone()
        n = cc[:4].tolist()
        mk, ne, offs = eng.masks(o, n, 640, 640)
        return ne.tolist()

    def dd():
        return m.predict(x)

    def dev():
        eng.run(x)

    print(f"device-only replays: {t(dev):.1f} us/step; (a) run+sync {t(a):.1f}; (b) +clone {t(b):.1f}; "
          f"(c) +masks+sync {t(c):.1f}; (d) predict {t(dd):.1f}", flush=True)


if __name__ == "__main__":
    main()
