#!/usr/bin/env python3
"""Timing ablation of one conv config on chosen ops of a workload: every conv op pinned to `--cfg`, per-op replay
times with YM_HALO_DBG = 0 (full), 1 (no DMA), 2 (no MFMA / LDS reads), 3 (neither)."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)


def child(a):
    import torch
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(task=a.task, size=a.model, device="cuda:0", dtype="f16")
    eng = m.model.engine
    x = synthetic_batch(a.batch, 640, 1000, torch.device("cuda", 0))
    eng.run(x)
    base = eng.rt.get_op_cfg(a.batch, 640, 640)
    names = [op.name for op in eng.graph.ops]
    want = a.ops.split(",")
    out = []
    for cfg in [int(c) for c in a.cfg.split(",")]:
        eng.rt.set_op_cfg(a.batch, 640, 640, [cfg if op.kind == "conv" else -1 for op in eng.graph.ops])
        t = eng.profile_replay(x, reps=20)
        out.append((cfg, [round(t[names.index(o)] * 1e3, 2) for o in want]))
    eng.rt.set_op_cfg(a.batch, 640, 640, base)
    t = eng.profile_replay(x, reps=20)
    out.append(("tuned", [round(t[names.index(o)] * 1e3, 2) for o in want]))
    for c, v in out:
        print(os.environ.get("YM_HALO_DBG", "0"), c, v, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cfg", default="75")
    ap.add_argument("--ops", default="model.3,model.5,model.2.m.0.cv1,model.23.cv2.0.0,model.4.m.0.cv1")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--dbg", default="0,1,2,3", help="YM_HALO_DBG values: 1 no DMA, 2 no MFMA, 4 no table, "
                    "8 no stores, 16 no K loop")
    a = ap.parse_args()
    if a.child:
        return child(a)
    print("dbg cfg", a.ops)
    for dbg in a.dbg.split(","):
        subprocess.run([sys.executable, __file__, "--child"] + sys.argv[1:], env=dict(os.environ, YM_HALO_DBG=dbg),
                       check=True, timeout=300)


if __name__ == "__main__":
    main()
