#!/usr/bin/env python3
"""CPU emulation of the x3 plan's operand representation on the oracle (where its coordinate error comes from).

The x3 plan stores every activation and every conv weight as hi = fp16(v), lo = fp16(v - hi) and multiplies
hi·w_hi + lo·w_hi + hi·w_lo.  fp16 subnormals (|lo| < 2^-14) keep only an absolute precision of 2^-25, so a weight
of magnitude 0.03 is held to ~1e-6 relative instead of fp32's 6e-8.  This tool re-runs the oracle with those
representations switched on per operand (tools/f16_emulate.py's rounding hooks with the split instead of the fp16
rounding) and reports, against the all-fp32 oracle and against a float64 forward (the exact answer):

    python tools/x3_emulate.py s 8

Metric (pre-NMS): over anchors whose fp32 best class score exceeds 0.2, max |Δscore| and max |Δxyxy| px.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import f16_emulate as E  # noqa: E402
from oracle import yolo11 as Y  # noqa: E402

SCALE_W = {"on": False}


def split_repr(t):
    """hi + lo as the x3 kernels see it (fp16 subnormals kept, as v_mfma_f32_*_f16 does)."""
    if SCALE_W["on"] and t.dim() == 4 and t.shape[1] > 1 and t.shape[0] > 4:  # weights: per-tensor power-of-2 scale
        m = float(t.abs().max())
        s = 2.0 ** (14 - int(torch.tensor(m).log2().ceil()))
        ts = t * s
        hi = ts.half().float()
        return (hi + (ts - hi).half().float()) / s
    hi = t.half().float()
    return hi + (t - hi).half().float()


def main():
    from tests.golden.make_golden import make_input
    from yolomi.synth import synth_weights
    scale = sys.argv[1] if len(sys.argv) > 1 else "s"
    nimg = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.set_num_threads(8)
    sd = synth_weights(scale, "detect", 0)
    net = Y.build(scale, "detect", sd, fuse=True)
    ops = E.install(net)
    x = make_input("uniform", tuple(range(9000, 9000 + nimg)), 640)
    E.R.update(w=set(), a=set(), input=False, p=False)
    y32 = E.run(net, x)
    net64 = Y.build(scale, "detect", sd, fuse=True).double()
    with torch.no_grad():
        (y64, _), _ = net64(x.double())
    y64 = y64.float()
    print("fp32 oracle vs float64:", E.metric(y64, y32), flush=True)
    E.rnd = split_repr
    for name, w, a, sw in (("x3 weights+acts", True, True, False), ("x3 weights only", True, False, False),
                           ("x3 acts only", False, True, False), ("x3 acts + pow2-scaled weights", True, True, True)):
        SCALE_W["on"] = sw
        E.R.update(w=set(ops) if w else set(), a=set(ops) if a else set(), input=False, p=False)
        y = E.run(net, x)
        print(f"{name:32s} vs fp32 oracle {E.metric(y32, y)}  vs float64 {E.metric(y64, y)}", flush=True)


if __name__ == "__main__":
    main()
