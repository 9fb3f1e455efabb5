#!/usr/bin/env python3
"""Diagnose int8 GPU-vs-oracle differences: every stored tensor of the int8 plan against the oracle's trace, in plan
order; for the first mismatching conv output prints the oracle's pre-rounding values at the mismatches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import quant as Q  # noqa: E402
from tests.golden.make_golden import make_input  # noqa: E402
from yolomi.synth import synth_weights  # noqa: E402


def main(name):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", name + ".json")))
    qp = Q.qparams_from_json(g["qparams"])
    sd = synth_weights("n", "detect", 0)
    x = make_input("uniform", g["input"]["seeds"], g["input"]["size"])
    om = Q.Int8OracleModel("n", "detect", sd, qp)
    om.ctx.trace = {}
    om.raw(x)
    tr = om.ctx.trace
    from core.model import YOLO11Model
    m = YOLO11Model(task="detect", size="n", device="cuda:0", dtype="i8", qparams=qp)
    eng = m.model.engine
    eng.run(x.cuda(), use_graph=False)
    B = x.shape[0]
    shown = 0
    for op in eng.graph.ops:
        a = op.args
        dst = a.get("dst")
        if dst is None or not hasattr(dst, "buf"):
            continue
        b = dst.buf
        if not b.qname or b.f32:
            continue
        got = eng.read_buffer(b.id, B)[..., dst.coff:dst.coff + dst.C]
        ref = tr.get(b.qkey)
        if ref is None:
            print(op.name, "no oracle tensor for", b.qkey)
            continue
        r = ref.q.permute(0, 2, 3, 1)[..., dst.coff:dst.coff + dst.C]
        d = (got - r).abs()
        nbad = int((d > 0).sum())
        print(f"{op.name:28s} -> {b.qkey:34s} mismatches {nbad:8d} / {d.numel():9d} max {float(d.max()):.0f}")
        if nbad and shown < 2 and op.kind == "conv":
            shown += 1
            y = tr["y:" + a["wkey"]].permute(0, 2, 3, 1)
            so, zo = qp["out:" + a["wkey"]]
            idx = torch.nonzero(d > 0)[:8]
            for t in idx.tolist():
                bb, yy, xx, cc = t
                yv = float(y[bb, yy, xx, cc + 0])
                print("   at", t, "gpu", float(got[bb, yy, xx, cc]), "oracle", float(r[bb, yy, xx, cc]), "y", yv,
                      "y*inv_sc", yv * Q.inv32(so), "zo", zo)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "det_n_i8_qnnpack")
