#!/usr/bin/env python3
"""Phase ablations of the fused Bottleneck kernel (csrc/ym_conv_bneck.hip, YM_BNECK_DBG bits: 1 no input loads,
2 no cv1, 4 no cv2, 8 no stores): replay time of every fused Bottleneck op per variant.  One process per setting
(the kernel reads the variable once).  GPU only.

    python tools/bneck_ablate.py [--model s] [--cfgs 79-86] [--dbg 0,1,2,4,8,15]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(model, cfgs):
    sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
    sys.path.insert(0, ROOT)
    import torch
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(size=model, device="cuda:0", dtype="f16")
    e = m.model.engine
    x = synthetic_batch(8, 640, 1000, torch.device("cuda", 0))
    e.run(x)
    ops = e.graph.ops
    bn = [i for i, op in enumerate(ops) if op.args.get("pair") and (op.args["pair"]["k"] == 3 or op.args["s"] == 2)]
    base = e.rt.get_op_cfg(8, 640, 640)
    for c in cfgs:
        e.rt.set_op_cfg(8, 640, 640, [c if i in bn else base[i] for i in range(len(ops))])
        t = e.profile_replay(x, reps=20)
        print(f"cfg {c}: " + "  ".join(f"{ops[i].name.split('.cv')[0]} {t[i] * 1e3:6.1f}" for i in bn), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--cfgs", default="79-86")
    ap.add_argument("--dbg", default="0,1,2,4,8,15")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    lo, _, hi = a.cfgs.partition("-")
    cfgs = list(range(int(lo), int(hi or lo) + 1))
    if a.child:
        return child(a.model, cfgs)
    for d in a.dbg.split(","):
        print(f"YM_BNECK_DBG={d}", flush=True)
        r = subprocess.run([sys.executable, __file__, "--child", "--model", a.model, "--cfgs", a.cfgs],
                           env=dict(os.environ, YM_BNECK_DBG=d), timeout=300)
        if r.returncode:
            return r.returncode


if __name__ == "__main__":
    sys.exit(main() or 0)
