"""Sweep the conv tile configurations (ym_set_debug YM_DBG_CONV_CFG) and report per-layer device time for each.

    python -m yolomi.tune --model n --batch 8
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7,8")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args(argv)
    os.environ["YM_AUTOTUNE"] = "0"
    from . import lib as L
    from .engine import Engine
    from .synth import synth_weights, uniform
    dev = torch.device("cuda", 0)
    eng = Engine(a.model, "detect", synth_weights(a.model, "detect", 0), dev, a.dtype)
    B, S = a.batch, a.size
    x = torch.from_numpy(uniform(5, B * 3 * S * S).astype(np.float32).reshape(B, 3, S, S)).to(dev)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    res = {}
    for c in [-1] + cfgs:
        L.set_debug(L.DBG_CONV_CFG, c + 1)  # (value + 1; 0: the heuristic)
        eng.profile(x)
        t = np.zeros(len(eng.graph.ops))
        for _ in range(a.reps):
            t += np.array(eng.profile(x))
        res[c] = t / a.reps
    L.set_debug(L.DBG_CONV_CFG, 0)
    conv = [i for i, op in enumerate(eng.graph.ops) if op.kind == "conv"]
    print("op | M N K | heuristic " + " ".join(f"c{c:>5}" for c in cfgs) + " | best")
    best_sum, heur_sum = 0.0, 0.0
    for i in conv:
        op = eng.graph.ops[i]
        ar = op.args
        fo = eng.graph.out_factor(op)
        M = B * (S // fo) ** 2
        row = [res[c][i] * 1e3 for c in cfgs]
        b = int(np.argmin(row))
        best_sum += row[b]
        heur_sum += res[-1][i] * 1e3
        print(f"{op.name:26s} k{ar['k']}s{ar['s']} {M:7d} {ar['c2']:4d} {ar['k'] ** 2 * ar['c1']:5d} | "
              f"{res[-1][i] * 1e3:7.1f} " + " ".join(f"{v:7.1f}" for v in row) + f" | c{cfgs[b]}")
    print(f"conv total (us): heuristic {heur_sum:.1f}  per-layer best {best_sum:.1f}")
    from .lib import Runtime
    args = Runtime.make_args(use_graph=False)
    dets, counts = eng.outputs(B, 300)
    st = torch.cuda.current_stream().cuda_stream
    eng.rt.tune(x.data_ptr(), B, S, S, args, dets.data_ptr(), counts.data_ptr(), st)
    cfg = eng.rt.get_op_cfg(B, S, S)
    t = np.zeros(len(eng.graph.ops))
    for _ in range(a.reps):
        t += np.array(eng.profile(x))
    t /= a.reps
    print("autotuned cfgs:", [cfg[i] for i in conv])
    print(f"conv total (us) with autotuned cfgs (eager events): {sum(t[i] for i in conv) * 1e3:.1f}")


if __name__ == "__main__":
    main()
