#!/usr/bin/env python3
"""Forward time vs confidence threshold (the validator's conf 0.001 vs predict's 0.25): graph-replayed forwards of
yolo11s x3 B=8 on the bench batch, events around 20 replays per threshold; the detections kept per image.  GPU only.

    CONFS=0.001 python tools/conf_timing.py [scale] [B]     (CONFS: the thresholds, default 0.25,0.05,0.01,0.001)"""
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
    m = YOLO11Model(task="detect", size=scale, device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    x = synthetic_batch(B, 640, 1000, torch.device("cuda", 0))
    for conf in [float(c) for c in os.environ.get("CONFS", "0.25,0.05,0.01,0.001").split(",")]:
        for _ in range(3):
            eng.run(x, conf=conf)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            d, c = eng.run(x, conf=conf)
        e1.record()
        torch.cuda.synchronize()
        print(f"conf {conf}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us per forward, kept {c[:B].tolist()}", flush=True)


if __name__ == "__main__":
    main()
