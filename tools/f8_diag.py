#!/usr/bin/env python3
"""fp8 plan diagnosis: layer-local agreement of plain Conv layers (model.1, 3, 5, 7) between the GPU and the fp8
oracle fed the GPU's own stored input, with variants of the oracle's arithmetic (subnormal e4m3 inputs / weights
flushed to zero, fp32 instead of float64 accumulation) to find which matches the fp8 MFMA."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import json  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    from core.model import YOLO11Model
    from oracle import quant as Q
    from tests.golden.make_golden import make_input
    from yolomi.synth import synth_weights
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "det_n_f8.json")))
    qp = Q.qparams_from_json(g["qparams"])
    m = YOLO11Model(task="detect", size="n", device="cuda:0", dtype="f8", qparams=qp)
    eng = m.model.engine
    x = make_input("uniform", g["input"]["seeds"], g["input"]["size"])
    eng.run(x.cuda(), use_graph=False)
    net = Q.build_folded("n", "detect", synth_weights("n", "detect", 0))
    mods = dict(net.named_modules())
    bufs = {b.name: b for b in eng.graph.buffers}
    cfg = eng.rt.get_op_cfg(2, 640, 640)
    names = [op.name for op in eng.graph.ops]
    from oracle.predict import OracleModel
    from yolomi.metrics import evaluate
    om = OracleModel("n", "detect", synth_weights("n", "detect", 0))
    fl = [r["boxes"].numpy() for r in om.predict(x)]
    o8 = [np.array(d, np.float32).reshape(-1, 6) for d in g["dets"]]
    g8 = [r.boxes.data.cpu().numpy() for r in m.predict(x.cuda())]
    print("mAP fp8-oracle vs float", evaluate(o8, fl), "gpu-f8 vs float", evaluate(g8, fl), "gpu-f8 vs fp8-oracle",
          evaluate(g8, o8), "counts", [len(a) for a in o8], [len(a) for a in g8], [len(a) for a in fl], flush=True)
    for i in (1, 3, 5, 7):
        src = eng.read_buffer(bufs[f"L{i - 1}"].id, 2)[..., :bufs[f"L{i - 1}"].C].permute(0, 3, 1, 2).contiguous()
        got = eng.read_buffer(bufs[f"L{i}"].id, 2)[..., :bufs[f"L{i}"].C].permute(0, 3, 1, 2).contiguous()
        conv = mods[f"model.{i}"].conv
        wq, sw = Q.quantize_weight_fp8(conv.weight)
        s_in = qp[f"act:model.{i - 1}"][0]
        so = qp[f"out:model.{i}"][0]
        s_b = qp[f"act:model.{i}"][0]
        sasw = (Q._t32(s_in) * torch.from_numpy(sw)).view(1, -1, 1, 1)
        sub = 2.0 ** -6
        for tag, xin, w, acc_dt in (("exact", src, wq, torch.float64),
                                    ("ftz-in", torch.where(src.abs() < sub, 0.0, src), wq, torch.float64),
                                    ("ftz-w", src, torch.where(wq.abs() < sub, 0.0, wq), torch.float64),
                                    ("ftz-both", torch.where(src.abs() < sub, 0.0, src),
                                     torch.where(wq.abs() < sub, 0.0, wq), torch.float64),
                                    ("fp32-acc", src, wq, torch.float32)):
            acc = F.conv2d(xin.to(acc_dt), w.to(acc_dt), None, conv.stride, conv.padding).float()
            y = acc * sasw + conv.bias.detach().float().view(1, -1, 1, 1)
            post = Q.silu64(Q.quantize_fp8(y, so) * Q._t32(so))
            ref = Q.quantize_fp8(post, s_b)
            same = float((ref == got).float().mean())
            grid = torch.unique(torch.arange(256).to(torch.uint8).view(torch.float8_e4m3fn).float().nan_to_num(0.0))
            dist = (torch.searchsorted(grid, ref.flatten()) - torch.searchsorted(grid, got.flatten())).abs()
            print(f"model.{i} cfg {cfg[names.index(f'model.{i}')]} {tag:9s} exact codes {same:.6f} "
                  f"max code distance {int(dist.max())} (>1: {int((dist > 1).sum())})", flush=True)


if __name__ == "__main__":
    main()
