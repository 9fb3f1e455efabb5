"""Restatement of the Ultralytics YOLO11 module tree in plain torch (CPU, fp32). TEST INFRASTRUCTURE ONLY.

Upstream (not in /root/reference, not installed): ultralytics 8.3.x `nn/modules/{conv,block,head}.py`,
`nn/tasks.py:parse_model`.  Reached from the reference at `core/model.py:110` (`YOLO(model_path)`) and
`core/model.py:133` (`self.model.predict`).  Module names follow Ultralytics so an Ultralytics-style state dict
(`model.{i}.cv1.conv.weight`, ...) loads with strict=True.
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

SCALES = {"n": (0.50, 0.25, 1024), "s": (0.50, 0.50, 1024), "m": (0.50, 1.00, 512), "l": (1.00, 1.00, 512),
          "x": (1.00, 1.50, 512)}


def _autopad(k: int) -> int:
    return k // 2


class Conv(nn.Module):
    """conv2d(bias=False) → BatchNorm2d(eps=1e-3) → SiLU (ultralytics `Conv`)."""

    def __init__(self, c1, c2, k=1, s=1, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, _autopad(k), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3, momentum=0.03)  # Ultralytics initialize_weights sets eps 1e-3
        self.act = nn.SiLU() if act else nn.Identity()
        self.fused = False

    @torch.no_grad()
    def fuse(self):
        """ultralytics `fuse_conv_and_bn`: W' = diag(γ/√(σ²+eps))·W, b' = β − γ·μ/√(σ²+eps)."""
        conv, bn = self.conv, self.bn
        fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                          groups=conv.groups, bias=True).requires_grad_(False)
        w_conv = conv.weight.view(conv.out_channels, -1)
        w_bn = torch.diag(bn.weight.div(torch.sqrt(bn.eps + bn.running_var)))
        fused.weight.copy_(torch.mm(w_bn, w_conv).view(fused.weight.shape))
        b_conv = torch.zeros(conv.weight.shape[0])
        b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
        fused.bias.copy_(torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn)
        self.conv = fused
        del self.bn
        self.fused = True

    def forward(self, x):
        if self.fused:
            return self.act(self.conv(x))
        return self.act(self.bn(self.conv(x)))


class DWConv(Conv):
    def __init__(self, c1, c2, k=1, s=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), act=act)


class Bottleneck(nn.Module):
    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        return x + self.cv2(self.cv1(x)) if self.add else self.cv2(self.cv1(x))


class C2f(nn.Module):
    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=(3, 3), e=1.0) for _ in range(n))

    def forward(self, x):
        y = list(self.cv1(x).chunk(2, 1))
        y.extend(m(y[-1]) for m in self.m)
        return self.cv2(torch.cat(y, 1))


class C3(nn.Module):
    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=(1, 3), e=1.0) for _ in range(n)))

    def forward(self, x):
        return self.cv3(torch.cat((self.m(self.cv1(x)), self.cv2(x)), 1))


class C3k(C3):
    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k=3):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=(k, k), e=1.0) for _ in range(n)))


class C3k2(C2f):
    def __init__(self, c1, c2, n=1, c3k=False, e=0.5, g=1, shortcut=True):
        super().__init__(c1, c2, n, shortcut, g, e)
        self.m = nn.ModuleList(C3k(self.c, self.c, 2, shortcut, g) if c3k else Bottleneck(self.c, self.c, shortcut, g)
                               for _ in range(n))


class SPPF(nn.Module):
    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(kernel_size=k, stride=1, padding=k // 2)

    def forward(self, x):
        y = [self.cv1(x)]
        y.extend(self.m(y[-1]) for _ in range(3))
        return self.cv2(torch.cat(y, 1))


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, attn_ratio=0.5):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.key_dim = int(self.head_dim * attn_ratio)
        self.scale = self.key_dim ** -0.5
        nh_kd = self.key_dim * num_heads
        h = dim + nh_kd * 2
        self.qkv = Conv(dim, h, 1, act=False)
        self.proj = Conv(dim, dim, 1, act=False)
        self.pe = Conv(dim, dim, 3, 1, g=dim, act=False)

    def forward(self, x):
        B, C, H, W = x.shape
        N = H * W
        qkv = self.qkv(x)
        q, k, v = qkv.view(B, self.num_heads, self.key_dim * 2 + self.head_dim, N).split(
            [self.key_dim, self.key_dim, self.head_dim], dim=2)
        attn = (q.transpose(-2, -1) @ k) * self.scale
        attn = attn.softmax(dim=-1)
        x = (v @ attn.transpose(-2, -1)).view(B, C, H, W) + self.pe(v.reshape(B, C, H, W))
        return self.proj(x)


class PSABlock(nn.Module):
    def __init__(self, c, attn_ratio=0.5, num_heads=4, shortcut=True):
        super().__init__()
        self.attn = Attention(c, attn_ratio=attn_ratio, num_heads=num_heads)
        self.ffn = nn.Sequential(Conv(c, c * 2, 1), Conv(c * 2, c, 1, act=False))
        self.add = shortcut

    def forward(self, x):
        x = x + self.attn(x) if self.add else self.attn(x)
        x = x + self.ffn(x) if self.add else self.ffn(x)
        return x


class C2PSA(nn.Module):
    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__()
        assert c1 == c2
        self.c = int(c1 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv(2 * self.c, c1, 1)
        self.m = nn.Sequential(*(PSABlock(self.c, attn_ratio=0.5, num_heads=self.c // 64) for _ in range(n)))

    def forward(self, x):
        a, b = self.cv1(x).split((self.c, self.c), dim=1)
        b = self.m(b)
        return self.cv2(torch.cat((a, b), 1))


class Concat(nn.Module):
    def forward(self, xs):
        return torch.cat(xs, 1)


class DFL(nn.Module):
    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1

    def forward(self, x):
        b, _, a = x.shape
        return self.conv(x.view(b, 4, self.c1, a).transpose(2, 1).softmax(1)).view(b, 4, a)


def make_anchors(feats, strides, offset=0.5):
    pts, st = [], []
    for i, s in enumerate(strides):
        h, w = feats[i].shape[2:]
        sx = torch.arange(w, dtype=feats[0].dtype) + offset
        sy = torch.arange(h, dtype=feats[0].dtype) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), s, dtype=feats[0].dtype))
    return torch.cat(pts), torch.cat(st)


def dist2bbox(distance, anchor_points, xywh=True, dim=-1):
    lt, rb = distance.chunk(2, dim)
    x1y1 = anchor_points - lt
    x2y2 = anchor_points + rb
    if xywh:
        return torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), dim)
    return torch.cat((x1y1, x2y2), dim)


class Detect(nn.Module):
    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc, self.nl, self.reg_max = nc, len(ch), 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.tensor([8.0, 16.0, 32.0])
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1))
                                 for x in ch)
        self.cv3 = nn.ModuleList(nn.Sequential(nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                                               nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)),
                                               nn.Conv2d(c3, self.nc, 1)) for x in ch)
        self.dfl = DFL(self.reg_max)

    def forward(self, x):
        for i in range(self.nl):
            x[i] = torch.cat((self.cv2[i](x[i]), self.cv3[i](x[i])), 1)
        return self._inference(x), x

    def _inference(self, x):
        shape = x[0].shape
        x_cat = torch.cat([xi.view(shape[0], self.no, -1) for xi in x], 2)
        anchors, strides = (t.transpose(0, 1) for t in make_anchors(x, self.stride, 0.5))
        box, cls = x_cat.split((self.reg_max * 4, self.nc), 1)
        dbox = dist2bbox(self.dfl(box), anchors.unsqueeze(0), xywh=True, dim=1) * strides
        return torch.cat((dbox, cls.sigmoid()), 1)


class Proto(nn.Module):
    def __init__(self, c1, c_=256, c2=32):
        super().__init__()
        self.cv1 = Conv(c1, c_, k=3)
        self.upsample = nn.ConvTranspose2d(c_, c_, 2, 2, 0, bias=True)
        self.cv2 = Conv(c_, c_, k=3)
        self.cv3 = Conv(c_, c2)

    def forward(self, x):
        return self.cv3(self.cv2(self.upsample(self.cv1(x))))


class Segment(Detect):
    def __init__(self, nc=80, nm=32, npr=256, ch=()):
        super().__init__(nc, ch)
        self.nm, self.npr = nm, npr
        self.proto = Proto(ch[0], self.npr, self.nm)
        c4 = max(ch[0] // 4, self.nm)
        self.cv4 = nn.ModuleList(nn.Sequential(Conv(x, c4, 3), Conv(c4, c4, 3), nn.Conv2d(c4, self.nm, 1)) for x in ch)

    def forward(self, x):
        p = self.proto(x[0])
        bs = p.shape[0]
        mc = torch.cat([self.cv4[i](x[i]).view(bs, self.nm, -1) for i in range(self.nl)], 2)
        y, feats = Detect.forward(self, x)
        return torch.cat([y, mc], 1), (feats, mc, p)


class Upsample(nn.Module):
    def forward(self, x):
        return F.interpolate(x, scale_factor=2.0, mode="nearest")


def _md(x, d=8):
    return int(math.ceil(x / d) * d)


class YOLO11(nn.Module):
    """DetectionModel / SegmentationModel for the yolo11{n,s,m,l,x}{,-seg} yaml."""

    def __init__(self, scale="n", task="detect", nc=80):
        super().__init__()
        depth, width, mc = SCALES[scale]
        ch = lambda c: _md(min(c, mc) * width, 8)  # noqa: E731
        rep = lambda n: max(round(n * depth), 1) if n > 1 else n  # noqa: E731
        c3k_force = scale in "mlx"
        L = []
        L.append(Conv(3, ch(64), 3, 2))
        L.append(Conv(ch(64), ch(128), 3, 2))
        L.append(C3k2(ch(128), ch(256), rep(2), c3k_force or False, 0.25))
        L.append(Conv(ch(256), ch(256), 3, 2))
        L.append(C3k2(ch(256), ch(512), rep(2), c3k_force or False, 0.25))
        L.append(Conv(ch(512), ch(512), 3, 2))
        L.append(C3k2(ch(512), ch(512), rep(2), True))
        L.append(Conv(ch(512), ch(1024), 3, 2))
        L.append(C3k2(ch(1024), ch(1024), rep(2), True))
        L.append(SPPF(ch(1024), ch(1024), 5))
        L.append(C2PSA(ch(1024), ch(1024), rep(2)))
        L.append(Upsample())
        L.append(Concat())
        L.append(C3k2(ch(1024) + ch(512), ch(512), rep(2), c3k_force or False))
        L.append(Upsample())
        L.append(Concat())
        L.append(C3k2(ch(512) + ch(512), ch(256), rep(2), c3k_force or False))
        L.append(Conv(ch(256), ch(256), 3, 2))
        L.append(Concat())
        L.append(C3k2(ch(256) + ch(512), ch(512), rep(2), c3k_force or False))
        L.append(Conv(ch(512), ch(512), 3, 2))
        L.append(Concat())
        L.append(C3k2(ch(512) + ch(1024), ch(1024), rep(2), True))
        heads = [ch(256), ch(512), ch(1024)]
        if task == "segment":
            L.append(Segment(nc, 32, _md(min(256, mc) * width, 8), heads))
        else:
            L.append(Detect(nc, heads))
        self.model = nn.Sequential(*L)
        self.task = task
        self.froms = {12: (-1, 6), 15: (-1, 4), 18: (-1, 13), 21: (-1, 10), 23: (16, 19, 22)}

    def fuse(self):
        for m in self.modules():
            if isinstance(m, Conv) and not m.fused:
                m.fuse()
        return self

    def forward(self, x, keep=()):
        """DetectionModel._predict_once; `keep` = layer indices whose outputs are also returned (bisecting)."""
        y: List = []
        saved = {}
        for i, m in enumerate(self.model):
            if i in self.froms:
                x = [x if j == -1 else y[j] for j in self.froms[i]]
            x = m(x)
            y.append(x)
            if i in keep:
                saved[i] = x
        return x, saved


def build(scale="n", task="detect", state_dict=None, fuse=True) -> YOLO11:
    m = YOLO11(scale, task).eval().requires_grad_(False)
    if state_dict is not None:
        sd = {k: torch.as_tensor(v) for k, v in state_dict.items()}
        m.load_state_dict(sd, strict=True)
    if fuse:
        m.fuse()
    return m.requires_grad_(False)
