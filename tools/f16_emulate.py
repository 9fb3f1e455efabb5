#!/usr/bin/env python3
"""CPU emulation of the f16 plan's rounding points on the oracle, op by op (precision budget).

The GPU f16 plan computes every conv as an fp32-accumulated GEMM of fp16 operands: the folded weights are rounded to
fp16, every stored activation is rounded to fp16 (after bias, SiLU and the residual add of the epilogue), the stem
reads the fp32 input into an fp16 patch, the attention kernel rounds the softmax probabilities to fp16 for the PV
MFMA, and the Detect rows are stored fp32.  This tool reproduces those rounding points on the torch-CPU oracle with a
per-op switch, so the error each op contributes to the boxes and scores can be measured without a GPU:

    python tools/f16_emulate.py s            # per-op sensitivity table + greedy promotion set

Metric (pre-NMS, a superset of what NMS keeps): over every anchor whose fp32 max class score exceeds 0.2, the max
|Δscore| of its best class and the max |Δ| of its xyxy box (px), against the all-fp32 oracle.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import yolo11 as Y  # noqa: E402

# ---------------------------------------------------------------------------------------------- rounding switches
R = {"w": set(), "a": set(), "input": False, "p": False}  # op names whose weights / stored outputs are rounded


def rnd(t):
    return t.half().float()


def _conv_fwd(self, x):
    w, b = self.conv.weight, self.conv.bias
    if self._n in R["w"]:
        w = rnd(w)
    y = F.conv2d(x, w, b, self.conv.stride, self.conv.padding, 1, self.conv.groups)
    y = self.act(y)
    if self._n in R["a"] and not getattr(self, "_res", False):
        y = rnd(y)
    return y


def _plain_fwd(self, x):  # Detect / Segment final nn.Conv2d (fp32 rows; fp16 weights)
    w = rnd(self.weight) if self._n in R["w"] else self.weight
    return F.conv2d(x, w, self.bias)


def _bneck_fwd(self, x):
    y = self.cv2(self.cv1(x))
    if not self.add:
        return y
    y = x + y
    return rnd(y) if self.cv2._n in R["a"] else y


def _attn_fwd(self, x):
    B, C, H, W = x.shape
    N = H * W
    qkv = self.qkv(x)
    q, k, v = qkv.view(B, self.num_heads, self.key_dim * 2 + self.head_dim, N).split(
        [self.key_dim, self.key_dim, self.head_dim], dim=2)
    attn = ((q.transpose(-2, -1) @ k) * self.scale).softmax(dim=-1)
    if R["p"]:
        attn = rnd(attn)
    y = (v @ attn.transpose(-2, -1)).view(B, C, H, W) + self.pe(v.reshape(B, C, H, W))
    if self._n in R["a"]:
        y = rnd(y)
    return self.proj(y)


def _psa_fwd(self, x):
    x = x + self.attn(x)
    if self.attn.proj._n in R["a"]:
        x = rnd(x)
    x = x + self.ffn(x)
    if self.ffn[1]._n in R["a"]:
        x = rnd(x)
    return x


def install(net):
    """Name every op like the GPU plan (GraphBuilder op names) and patch the forwards."""
    names = []
    for name, m in net.named_modules():
        if isinstance(m, Y.Conv):
            m._n = name
            m.forward = _conv_fwd.__get__(m)
            names.append(name)
        elif (isinstance(m, torch.nn.Conv2d) and not name.endswith(".conv") and ".dfl" not in name
              and ".proto" not in name):
            m._n = name
            m.forward = _plain_fwd.__get__(m)
            names.append(name)
        if isinstance(m, Y.Bottleneck):
            m.forward = _bneck_fwd.__get__(m)
            if m.add:
                m.cv2._res = True
        if isinstance(m, Y.Attention):
            m._n = name
            m.forward = _attn_fwd.__get__(m)
            m.pe._res = True   # pe(v) is added to the attention output before the one rounding
            m.proj._res = True
            names.append(name)
        if isinstance(m, Y.PSABlock):
            m.forward = _psa_fwd.__get__(m)
            m.ffn[1]._res = True
    return names


def run(net, x):
    with torch.no_grad():
        xi = rnd(x) if R["input"] else x
        (y, _), _ = net(xi)
    return y


def metric(y_ref, y, thr=0.2):
    """(max |Δscore|, max |Δxyxy| px, rms Δscore, rms Δxyxy) over anchors with ref best score > thr."""
    nc = 80
    box_r, cls_r = y_ref[:, :4], y_ref[:, 4:4 + nc]
    box_g, cls_g = y[:, :4], y[:, 4:4 + nc]
    sc, j = cls_r.max(1)                          # (B, A)
    m = sc > thr
    sg = cls_g.gather(1, j[:, None]).squeeze(1)
    ds = (sg - sc).abs()[m]

    def xyxy(b):
        return torch.cat([b[:, :2] - b[:, 2:] / 2, b[:, :2] + b[:, 2:] / 2], 1)
    db = (xyxy(box_g) - xyxy(box_r)).abs().amax(1)[m]
    return (float(ds.max()), float(db.max()), float(ds.pow(2).mean().sqrt()), float(db.pow(2).mean().sqrt()))


def main():
    from tests.golden.make_golden import make_input
    from yolomi.synth import synth_weights
    scale = sys.argv[1] if len(sys.argv) > 1 else "s"
    nimg = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    torch.set_num_threads(8)
    net = Y.build(scale, "detect", synth_weights(scale, "detect", 0), fuse=True)
    ops = install(net)
    x = make_input("uniform", tuple(range(9000, 9000 + nimg)), 640)
    R.update(w=set(), a=set(), input=False, p=False)
    y_ref = run(net, x)
    out = {"ops": ops}

    def full(w=True, a=True, inp=True, p=True, skip=()):
        R.update(w=set(ops) - set(skip) if w else set(), a=set(ops) - set(skip) if a else set(), input=inp, p=p)
        return metric(y_ref, run(net, x))

    out["all_f16"] = full()
    out["weights_only"] = full(a=False, inp=False, p=False)
    out["acts_only"] = full(w=False)
    print("all f16", out["all_f16"], "weights only", out["weights_only"], "acts only", out["acts_only"], flush=True)
    # per-op: only this op rounded (weights + output)
    per = {}
    for n in ops:
        R.update(w={n}, a={n}, input=False, p=False)
        per[n] = metric(y_ref, run(net, x))
        print(f"{n:28s} max ds {per[n][0]:.2e} dxy {per[n][1]:.3f}  rms ds {per[n][2]:.2e} dxy {per[n][3]:.4f}",
              flush=True)
    out["per_op"] = per
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"f16_emulate_{scale}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
