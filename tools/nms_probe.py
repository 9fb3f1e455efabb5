#!/usr/bin/env python3
"""NMS cost vs candidate count: eager forwards of yolo11n B=8 at conf 0.99 / 0.5 / 0.25 / 0.1 (0, a few, ~10-140,
>300 candidates per image), for `rocprofv3 --kernel-trace` to time nms_image per call.  GPU only."""
import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "yolo-infer_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from bench import synthetic_batch
from core.model import YOLO11Model
m = YOLO11Model(size="n", device="cuda:0", dtype="f16", verbose=False)
eng = m.model.engine
x = synthetic_batch(8, 640, 1000, torch.device("cuda", 0))
for conf in [float(c) for c in os.environ.get("NMS_CONFS", "0.99,0.5,0.25,0.1").split(",")]:
    for _ in range(20):
        eng.run(x, conf=conf, use_graph=False)
    torch.cuda.synchronize()
    print("conf", conf, eng.run(x, conf=conf)[1].tolist(), flush=True)
