#!/usr/bin/env python3
"""NMS phase ablation on the bench workload (yolo11s B=8 x3, conf 0.25): per-op event time of nms_image with
YM_NMS_DBG=d (exit after phase d of the bit-matrix path; 6 = right after launch, 7 = after the count read; 0 = the
whole kernel), the median of 30 eager forwards, plus the per-image candidate counts.  One process per d (the
variable is read once per process):  for d in 0 1 2 3 4 5 6 7; do YM_NMS_DBG=$d python tools/nms_phases.py; done"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import synthetic_batch  # noqa: E402
from core.model import YOLO11Model  # noqa: E402

m = YOLO11Model(size=os.environ.get("NMS_MODEL", "s"), device="cuda:0", dtype=os.environ.get("NMS_DT", "x3"),
                verbose=False)
eng = m.model.engine
x = synthetic_batch(8, 640, 1000, torch.device("cuda", 0))
i = [k for k, op in enumerate(eng.graph.ops) if op.kind == "nms"][0]
j = [k for k, op in enumerate(eng.graph.ops) if op.kind == "decode"][0]
ts, td = [], []
for _ in range(30):
    t = eng.profile(x)
    ts.append(t[i] * 1e3)
    td.append(t[j] * 1e3)
cand = None
try:
    import numpy as np
    eng.run(x, use_graph=False)
    torch.cuda.synchronize()
except Exception:
    pass
print(f"YM_NMS_DBG={os.environ.get('YM_NMS_DBG', '0')}: nms {statistics.median(ts):.2f} us, decode "
      f"{statistics.median(td):.2f} us, kept {eng.run(x)[1].tolist()}", flush=True)
