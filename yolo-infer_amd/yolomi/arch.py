"""YOLO11 graph → flat NHWC execution plan for the HIP runtime.

This is the MI355X-side description of the graph the reference reaches through `ultralytics.YOLO(...)`
(`core/model.py:106-110`; architecture restated in SURVEY Appendix A).  It is *not* a module tree: it is a list of
fused kernel launches over channel-sliced NHWC buffers:

* every `Conv` (conv2d → BN → SiLU) is one implicit-GEMM launch with BN folded into weight/bias
  (Ultralytics `fuse_conv_and_bn`, eps 1e-3) and the activation, Bottleneck residual add and concat placement done
  in the epilogue (producers write straight into a channel slice of the concat buffer: no cat kernels);
* `Upsample(2, nearest)` + `Concat` never materialise: the consumer conv gets two A-sources, the first read at
  (y>>1, x>>1) (`up` flag);
* SPPF's three cascaded MaxPool2d(5,1,2) are one kernel writing three slices (max5∘max5 = max9, max5∘max5∘max5 =
  max13 exactly, with -inf padding);
* C2PSA's attention + positional depthwise conv is one kernel; `proj`/`ffn` residuals are conv epilogues;
* the Detect head's final 1x1 convs write fp32 straight into an anchor-major (B, A, no) buffer, which the decode
  and NMS kernels consume.

The same walk also enumerates every parameter with its Ultralytics state-dict name and shape, so synthetic weights
(`yolomi.synth`) and real checkpoints pack the same way.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

# scale → (depth, width, max_channels); SURVEY Appendix A parse rules
SCALES = {
    "n": (0.50, 0.25, 1024),
    "s": (0.50, 0.50, 1024),
    "m": (0.50, 1.00, 512),
    "l": (1.00, 1.00, 512),
    "x": (1.00, 1.50, 512),
}

NC = 80
REG_MAX = 16
STRIDES = (8, 16, 32)


def make_divisible(x: float, d: int = 8) -> int:
    return int(math.ceil(x / d) * d)


@dataclass
class Buffer:
    id: int
    C: int
    f: int            # spatial down-sampling factor w.r.t. the input (1, 2, ... 32); 0 = anchor-major buffer
    f32: bool = False  # storage fp32 regardless of activation dtype (head outputs)
    name: str = ""
    # int8 plans: the quantisation point of the tensor this buffer stores (oracle/quant.py naming): "act:<qname>" =
    # its own observer, "out:<qname>" = the output quantisation of the conv that writes it as is; None = float
    qname: Optional[str] = None
    qkind: str = "act"
    Cs: int = 0         # storage channels (row stride): C, or C rounded up to 16 in int8 plans

    @property
    def qkey(self) -> Optional[str]:
        return f"{self.qkind}:{self.qname}" if self.qname else None


@dataclass
class View:
    buf: Buffer
    coff: int
    C: int


@dataclass
class Op:
    kind: str
    args: Dict
    name: str = ""


@dataclass
class Param:
    name: str
    shape: Tuple[int, ...]
    kind: str
    extra: Dict = field(default_factory=dict)


class GraphBuilder:
    def __init__(self, scale: str = "n", task: str = "detect", nc: int = NC, quant: bool = False,
                 fuse=False):
        """quant=True builds the int8 (PTQ) plan: 16-channel storage granules and materialised concats (a concat is
        one quantized tensor with its own observer, so the two-source A loader is replaced by requant copies).
        fuse=True (f16 plans) merges each conv that feeds only a following 1x1 conv into one launch (fuse_pairs)
        and runs C3k's two 1x1 convs on the same input as one GEMM; fuse="merge" only the latter (a GEMM with the two
        weight matrices stacked along N: per output channel the same arithmetic as the two convs); fuse="x3" (x3
        plans) both, the conv → 1x1 pairs sized by the pair layout's doubled storage K (the streaming kernel's x3
        FUSE mode) and the Bottlenecks on conv_bneck's x3 mode."""
        if scale not in SCALES:
            raise ValueError(f"Unsupported size: {scale}")
        if task not in ("detect", "segment"):
            raise ValueError(f"task {task!r} has no HIP plan (supported: detect, segment)")
        self.scale, self.task, self.nc, self.quant = scale, task, nc, quant
        self.depth, self.width, self.max_ch = SCALES[scale]
        self.buffers: List[Buffer] = []
        self.ops: List[Op] = []
        self.params: List[Param] = []
        self.flops_per_pixel: List[Tuple[str, int, int]] = []  # (op name, factor, MACs per output pixel)
        self.fuse = bool(fuse)  # C3k cv1 ‖ cv2 merged
        self.x3 = fuse == "x3"  # pair-layout storage: fused pairs sized for it, 1x1 successors only
        self._build()
        if fuse is True or fuse == "x3":
            if quant:
                raise ValueError("fused conv pairs are f16-only (int8 plans requantise every conv output)")
            import os
            if self.x3 and os.environ.get("YM_FUSE_DW", "1") != "0":
                self.fuse_dw()
            self.fuse_pairs()

    # ------------------------------------------------------------------ helpers
    def ch(self, c: int) -> int:
        return make_divisible(min(c, self.max_ch) * self.width, 8)

    def rep(self, n: int) -> int:
        return max(round(n * self.depth), 1) if n > 1 else n

    def buf(self, C: int, f: int, name: str, f32: bool = False, q: Optional[str] = None, qkind: str = "act") -> Buffer:
        Cs = (C + 15) // 16 * 16 if (self.quant and not f32) else C
        b = Buffer(len(self.buffers), C, f, f32, name, None if f32 else q, qkind, Cs)
        self.buffers.append(b)
        return b

    def full(self, b: Buffer) -> View:
        return View(b, 0, b.C)

    def _conv_params(self, prefix: str, c1: int, c2: int, k: int, g: int = 1, bn: bool = True, bias_kind=None,
                     extra=None):
        w_kind = "conv_w" if bn else "head_w"
        self.params.append(Param(f"{prefix}.conv.weight" if bn else f"{prefix}.weight", (c2, c1 // g, k, k), w_kind))
        if bn:
            for suf, kind in (("weight", "bn_w"), ("bias", "bn_b"), ("running_mean", "bn_mean"),
                              ("running_var", "bn_var")):
                self.params.append(Param(f"{prefix}.bn.{suf}", (c2,), kind))
            self.params.append(Param(f"{prefix}.bn.num_batches_tracked", (), "count"))
        else:
            self.params.append(Param(f"{prefix}.bias", (c2,), bias_kind or "bias", extra or {}))

    def conv(self, prefix: str, src: View, c2: int, k: int, s: int, dst: View, act: bool = True,
             res: Optional[View] = None, src1: Optional[View] = None, up0: bool = False, bn: bool = True,
             bias_kind=None, extra=None, anchor_level: int = -1, shuffle2x2: bool = False,
             catq: Optional[str] = None):
        """catq: quantisation name of the concat a two-source conv reads (Ultralytics Concat module / cat tensor)."""
        c1 = src.C + (src1.C if src1 is not None else 0)
        self._conv_params(prefix, c1, c2, k, 1, bn, bias_kind, extra)
        assert dst.C == (4 * c2 if shuffle2x2 else c2) or anchor_level >= 0 or shuffle2x2
        fin = src.buf.f * (2 if s == 2 else 1) // (2 if up0 else 1)
        if self.quant and src1 is not None:  # int8: materialise the concat (requant copies into one tensor)
            f_in = src.buf.f // (2 if up0 else 1)
            cat = self.buf(c1, f_in, catq, q=catq)
            self.ops.append(Op("requant", dict(src=src, up=up0, dst=View(cat, 0, src.C)), catq + ".req0"))
            self.ops.append(Op("requant", dict(src=src1, up=False, dst=View(cat, src.C, src1.C)), catq + ".req1"))
            src, src1, up0 = self.full(cat), None, False
        self.ops.append(Op("conv", dict(k=k, s=s, c1=c1, c2=c2, act=act, src0=src, up0=up0, src1=src1, dst=dst,
                                        res=res, anchor_level=anchor_level, shuffle2x2=shuffle2x2, bn=bn,
                                        wkey=prefix, catq=catq), prefix))
        self.flops_per_pixel.append((prefix, fin, k * k * c1 * c2))

    def dwconv(self, prefix: str, src: View, dst: View, act: bool = True):
        C = src.C
        self._conv_params(prefix, C, C, 3, g=C)
        self.ops.append(Op("dwconv", dict(C=C, act=act, src=src, dst=dst, wkey=prefix), prefix))
        self.flops_per_pixel.append((prefix, src.buf.f, 9 * C))

    # ------------------------------------------------------------------ modules
    def Conv(self, i: int, x: View, c2: int, k: int, s: int) -> View:
        f = x.buf.f * s
        out = self.buf(c2, f, f"L{i}", q=f"model.{i}")
        self.conv(f"model.{i}", x, c2, k, s, self.full(out))
        return self.full(out)

    def bottleneck(self, prefix: str, x: View, c: int, e: float, dst: View, f: int):
        c_ = int(c * e)
        h = self.buf(c_, f, prefix + ".h", q=prefix + ".cv1")
        self.conv(prefix + ".cv1", x, c_, 3, 1, self.full(h))
        self.conv(prefix + ".cv2", self.full(h), c, 3, 1, dst, res=x)

    def c3k(self, prefix: str, x: View, c: int, dst: View, f: int, n: int = 2):
        c_ = int(c * 0.5)
        cat = self.buf(2 * c_, f, prefix + ".cat", q=prefix + ".cat")
        if self.fuse:
            # cv1 ‖ cv2 (both 1x1 on x) as one GEMM with N = 2c_: cv1's output lands in cat[0:c_], which nothing
            # reads after the first Bottleneck until the last one writes its output there; cv2's in cat[c_:2c_]
            self._conv_params(prefix + ".cv1", x.C, c_, 1)
            self._conv_params(prefix + ".cv2", x.C, c_, 1)
            self.ops.append(Op("conv", dict(k=1, s=1, c1=x.C, c2=2 * c_, act=True, src0=x, up0=False, src1=None,
                                            dst=self.full(cat), res=None, anchor_level=-1, shuffle2x2=False, bn=True,
                                            wkey=prefix + ".cv1", wkeys=[prefix + ".cv1", prefix + ".cv2"],
                                            catq=None), prefix + ".cv1+cv2"))
            self.flops_per_pixel.append((prefix + ".cv1+cv2", f, x.C * 2 * c_))
            cur = View(cat, 0, c_)
        else:
            t = self.buf(c_, f, prefix + ".t0", q=prefix + ".cv1")
            self.conv(prefix + ".cv1", x, c_, 1, 1, self.full(t))
            self.conv(prefix + ".cv2", x, c_, 1, 1, View(cat, c_, c_))
            cur = self.full(t)
        for j in range(n):
            last = j == n - 1
            nxt = View(cat, 0, c_) if last else self.full(self.buf(c_, f, f"{prefix}.t{j + 1}", q=f"{prefix}.m.{j}"))
            self.bottleneck(f"{prefix}.m.{j}", cur, c_, 1.0, nxt, f)
            cur = nxt
        self.conv(prefix + ".cv3", self.full(cat), c, 1, 1, dst)

    def C3k2(self, i: int, x: View, c2: int, n: int, c3k: bool, e: float, x1: Optional[View] = None,
             up0: bool = False) -> View:
        if self.scale in "mlx":
            c3k = True
        n = self.rep(n)
        f = x.buf.f // (2 if up0 else 1)
        c = int(c2 * e)
        cat = self.buf((2 + n) * c, f, f"L{i}.cat", q=f"model.{i}.cat")
        self.conv(f"model.{i}.cv1", x, 2 * c, 1, 1, View(cat, 0, 2 * c), src1=x1, up0=up0,
                  catq=f"model.{i - 1}" if x1 is not None else None)
        prev = View(cat, c, c)
        for j in range(n):
            dst = View(cat, (2 + j) * c, c)
            if c3k:
                self.c3k(f"model.{i}.m.{j}", prev, c, dst, f)
            else:
                self.bottleneck(f"model.{i}.m.{j}", prev, c, 0.5, dst, f)
            prev = dst
        out = self.buf(c2, f, f"L{i}", q=f"model.{i}")
        self.conv(f"model.{i}.cv2", self.full(cat), c2, 1, 1, self.full(out))
        return self.full(out)

    def SPPF(self, i: int, x: View, c2: int) -> View:
        c_ = x.C // 2
        f = x.buf.f
        cat = self.buf(4 * c_, f, f"L{i}.cat", q=f"model.{i}.cat")
        self.conv(f"model.{i}.cv1", x, c_, 1, 1, View(cat, 0, c_))
        self.ops.append(Op("sppf", dict(C=c_, src=View(cat, 0, c_), dst=cat), f"model.{i}.m"))
        out = self.buf(c2, f, f"L{i}", q=f"model.{i}")
        self.conv(f"model.{i}.cv2", self.full(cat), c2, 1, 1, self.full(out))
        return self.full(out)

    def C2PSA(self, i: int, x: View, c2: int, n: int) -> View:
        n = self.rep(n)
        f = x.buf.f
        c = int(x.C * 0.5)
        nh = c // 64
        hd = c // nh
        kd = int(hd * 0.5)
        h = c + 2 * nh * kd
        cv1 = self.buf(2 * c, f, f"L{i}.cv1", q=f"model.{i}.cv1")
        self.conv(f"model.{i}.cv1", x, 2 * c, 1, 1, self.full(cv1))
        b = View(cv1, c, c)
        for j in range(n):
            p = f"model.{i}.m.{j}"
            qkv = self.buf(h, f, p + ".qkv", q=p + ".attn.qkv", qkind="out")
            self.conv(p + ".attn.qkv", b, h, 1, 1, self.full(qkv), act=False)
            ao = self.buf(c, f, p + ".attn.o", q=p + ".attn.x")
            self._conv_params(p + ".attn.pe", c, c, 3, g=c)
            self.ops.append(Op("attn", dict(C=c, nh=nh, kd=kd, hd=hd, qkv=self.full(qkv), dst=self.full(ao),
                                            wkey=p + ".attn.pe"), p + ".attn"))
            self.flops_per_pixel.append((p + ".attn.pe", f, 9 * c))
            b1 = self.buf(c, f, p + ".b1", q=p + ".attn_add")
            self.conv(p + ".attn.proj", self.full(ao), c, 1, 1, self.full(b1), act=False, res=b)
            ff = self.buf(2 * c, f, p + ".ffn", q=p + ".ffn.0")
            self.conv(p + ".ffn.0", self.full(b1), 2 * c, 1, 1, self.full(ff))
            b2 = self.buf(c, f, p + ".b2", q=p)
            self.conv(p + ".ffn.1", self.full(ff), c, 1, 1, self.full(b2), act=False, res=self.full(b1))
            b = self.full(b2)
        out = self.buf(c2, f, f"L{i}", q=f"model.{i}")
        self.conv(f"model.{i}.cv2", View(cv1, 0, c), c2, 1, 1, self.full(out), src1=b, catq=f"model.{i}.cat")
        return self.full(out)

    def Detect(self, i: int, xs: List[View]):
        nc = self.nc
        no = nc + 4 * REG_MAX
        nm = 32 if self.task == "segment" else 0
        self.no, self.nm = no, nm
        anchor = self.buf(no + nm, 0, "anchors", f32=True)
        self.anchor_buf = anchor
        ch0 = xs[0].C
        c2 = max(16, ch0 // 4, REG_MAX * 4)
        c3 = max(ch0, min(nc, 100))
        p = f"model.{i}"
        if self.task == "segment":  # Proto on P3 (Segment.forward computes it first)
            npr = make_divisible(min(256, self.max_ch) * self.width, 8)
            f = xs[0].buf.f
            p1 = self.buf(npr, f, "proto.cv1", q=f"{p}.proto.cv1")
            self.conv(f"{p}.proto.cv1", xs[0], npr, 3, 1, self.full(p1))
            p2 = self.buf(npr, f // 2, "proto.up", q=f"{p}.proto.upsample", qkind="out")
            # ConvTranspose2d(npr, npr, 2, 2, bias): a 1x1 GEMM with N = 4*npr scattered 2x2 (pixel shuffle)
            self.params.append(Param(f"{p}.proto.upsample.weight", (npr, npr, 2, 2), "convT_w"))
            self.params.append(Param(f"{p}.proto.upsample.bias", (npr,), "bias"))
            self.ops.append(Op("conv", dict(k=1, s=1, c1=npr, c2=4 * npr, act=False, src0=self.full(p1), up0=False,
                                            src1=None, dst=self.full(p2), res=None, anchor_level=-1,
                                            shuffle2x2=True, bn=False, wkey=f"{p}.proto.upsample", convT=True,
                                            catq=None),
                               f"{p}.proto.upsample"))
            self.flops_per_pixel.append((f"{p}.proto.upsample", f, 4 * npr * npr))
            p3 = self.buf(npr, f // 2, "proto.cv2", q=f"{p}.proto.cv2")
            self.conv(f"{p}.proto.cv2", self.full(p2), npr, 3, 1, self.full(p3))
            proto = self.buf(nm, f // 2, "proto", f32=True)
            self.conv(f"{p}.proto.cv3", self.full(p3), nm, 1, 1, self.full(proto))
            self.proto_buf = proto
        for l, x in enumerate(xs):
            f = x.buf.f
            # box branch cv2: Conv(x,c2,3) → Conv(c2,c2,3) → Conv2d(c2, 64, 1)
            t1 = self.buf(c2, f, f"cv2.{l}.0", q=f"{p}.cv2.{l}.0")
            self.conv(f"{p}.cv2.{l}.0", x, c2, 3, 1, self.full(t1))
            t2 = self.buf(c2, f, f"cv2.{l}.1", q=f"{p}.cv2.{l}.1")
            self.conv(f"{p}.cv2.{l}.1", self.full(t1), c2, 3, 1, self.full(t2))
            self.conv(f"{p}.cv2.{l}.2", self.full(t2), 4 * REG_MAX, 1, 1, View(anchor, 0, 4 * REG_MAX),
                      act=False, bn=False, bias_kind="box_b", anchor_level=l)
            # cls branch cv3: [DWConv(x,x,3) → Conv(x,c3,1)] → [DWConv(c3,c3,3) → Conv(c3,c3,1)] → Conv2d(c3, nc, 1)
            d1 = self.buf(x.C, f, f"cv3.{l}.0.0", q=f"{p}.cv3.{l}.0.0")
            self.dwconv(f"{p}.cv3.{l}.0.0", x, self.full(d1))
            e1 = self.buf(c3, f, f"cv3.{l}.0.1", q=f"{p}.cv3.{l}.0.1")
            self.conv(f"{p}.cv3.{l}.0.1", self.full(d1), c3, 1, 1, self.full(e1))
            d2 = self.buf(c3, f, f"cv3.{l}.1.0", q=f"{p}.cv3.{l}.1.0")
            self.dwconv(f"{p}.cv3.{l}.1.0", self.full(e1), self.full(d2))
            e2 = self.buf(c3, f, f"cv3.{l}.1.1", q=f"{p}.cv3.{l}.1.1")
            self.conv(f"{p}.cv3.{l}.1.1", self.full(d2), c3, 1, 1, self.full(e2))
            self.conv(f"{p}.cv3.{l}.2", self.full(e2), nc, 1, 1, View(anchor, 4 * REG_MAX, nc), act=False,
                      bn=False, bias_kind="cls_b",
                      extra=dict(nc=nc, stride=STRIDES[l], shift=_cls_shift(self.scale)), anchor_level=l)
            if self.task == "segment":  # mask-coefficient branch cv4: Conv(x,c4,3) → Conv(c4,c4,3) → Conv2d(c4,nm,1)
                c4 = max(ch0 // 4, nm)
                m1 = self.buf(c4, f, f"cv4.{l}.0", q=f"{p}.cv4.{l}.0")
                self.conv(f"{p}.cv4.{l}.0", x, c4, 3, 1, self.full(m1))
                m2 = self.buf(c4, f, f"cv4.{l}.1", q=f"{p}.cv4.{l}.1")
                self.conv(f"{p}.cv4.{l}.1", self.full(m1), c4, 3, 1, self.full(m2))
                self.conv(f"{p}.cv4.{l}.2", self.full(m2), nm, 1, 1, View(anchor, no, nm), act=False, bn=False,
                          anchor_level=l)
        self.params.append(Param(f"{p}.dfl.conv.weight", (1, REG_MAX, 1, 1), "dfl"))
        self.ops.append(Op("decode", dict(anchor=anchor, nc=nc, nm=nm), f"{p}.decode"))
        self.ops.append(Op("nms", dict(nc=nc, nm=nm), f"{p}.nms"))

    # ------------------------------------------------------------------ the graph
    def _build(self):
        self.input = self.buf(8, 1, "input", q="input")  # RGB padded to 8 channels (16 B per pixel in fp16)
        self.ops.append(Op("input", dict(dst=self.input), "input"))
        x = View(self.input, 0, 3)
        ch = self.ch
        L0 = self.Conv(0, x, ch(64), 3, 2)
        L1 = self.Conv(1, L0, ch(128), 3, 2)
        L2 = self.C3k2(2, L1, ch(256), 2, False, 0.25)
        L3 = self.Conv(3, L2, ch(256), 3, 2)
        L4 = self.C3k2(4, L3, ch(512), 2, False, 0.25)
        L5 = self.Conv(5, L4, ch(512), 3, 2)
        L6 = self.C3k2(6, L5, ch(512), 2, True, 0.5)
        L7 = self.Conv(7, L6, ch(1024), 3, 2)
        L8 = self.C3k2(8, L7, ch(1024), 2, True, 0.5)
        L9 = self.SPPF(9, L8, ch(1024))
        L10 = self.C2PSA(10, L9, ch(1024), 2)
        # 11 Upsample + 12 Concat[-1, 6] fold into layer 13's cv1 (two-source A loader, first source up-sampled)
        L13 = self.C3k2(13, L10, ch(512), 2, False, 0.5, x1=L6, up0=True)
        L16 = self.C3k2(16, L13, ch(256), 2, False, 0.5, x1=L4, up0=True)
        L17 = self.Conv(17, L16, ch(256), 3, 2)
        L19 = self.C3k2(19, L17, ch(512), 2, False, 0.5, x1=L13)
        L20 = self.Conv(20, L19, ch(512), 3, 2)
        L22 = self.C3k2(22, L20, ch(1024), 2, True, 0.5, x1=L10)
        self.Detect(23, [L16, L19, L22])
        # the stem reads 3 real channels out of the 8-channel padded input: pad its weights' Cin to 8 at pack time

    # ------------------------------------------------------------------ fused pairs (f16 plans)
    STREAM_KS = {1: (2, 4, 6, 8), 3: (4, 6, 10, 18)}  # csrc/ym_conv_stream.hip K steps of 32 per kind
    DMA_FUSE_MAX = 128                               # csrc/ym_conv_dma.hip YM_DMA_FUSE_CFGS: BN <= 128 (x3 plans)
    FUSE_MAX_N = 128                                 # csrc/ym_conv_stream.hip kFuseMaxN
    FUSE_MAX_LDS = 112 * 1024                        # csrc/ym_conv_stream.hip kMaxFusedBytes

    def _readers(self, buf: Buffer) -> int:
        n = 0
        for op in self.ops:
            a = op.args
            views = [a.get(k) for k in ("src0", "src1", "res", "src", "qkv")]
            n += sum(1 for v in views if isinstance(v, View) and v.buf is buf)
            if op.kind == "sppf" and a["dst"] is buf:
                n += 1
        return n

    def fuse_pairs(self):
        """Merge conv A → 1x1 conv B when B immediately follows A and is the only reader of A's whole output
        buffer (the Detect/Segment head chains: cv2.l.1 → cv2.l.2, cv3.l.1.1 → cv3.l.2, cv4.l.1 → cv4.l.2).  The
        fused op runs A's conv, rounds its activated output to fp16 like the stored tensor, and multiplies it by
        B's weights in the same streaming kernel (csrc/ym_conv_stream.hip FUSE); A's output buffer is never
        written.  Same arithmetic as the unfused pair up to fp32 summation order in B."""
        out: List[Op] = []
        i = 0
        while i < len(self.ops):
            op = self.ops[i]
            nxt = self.ops[i + 1] if i + 1 < len(self.ops) else None
            if nxt is not None and self._fusable(op, nxt):
                a, b = op.args, nxt.args
                args = dict(a)
                args.update(dst=b["dst"], res=b["res"], anchor_level=b["anchor_level"],
                            pair=dict(k=b["k"], c1=b["c1"], c2=b["c2"], act=b["act"], bn=b["bn"], wkey=b["wkey"],
                                      dst=b["dst"], res=b["res"], mid=a["dst"]))
                out.append(Op("conv", args, f"{op.name}+{nxt.name.rsplit('.', 1)[-1]}"))
                i += 2
                continue
            out.append(op)
            i += 1
        self.ops = out

    DW_MAX_C, DW_MAX_N = 512, 128  # csrc/ym_conv_dwpw.hip kDwpwMaxC, 16 * kDwpwNB
    # map strides whose depthwise ops are fused: measured (yolo11s B=8 x3 replay, r04) the fused kernel beats the
    # depthwise + 1x1 launches on the P3 maps only (80²: 32.6 vs 35.5 us per pair); on P4 / P5 (40², 20²) the few
    # workgroups run their K blocks' load → depthwise → MFMA chains at ~2-4 us each and lose (21.8 vs 18.5 us,
    # 35.7 vs 14.9 us for the 512-channel P5 input).  Round 5 split those K blocks over 2-8 workgroups (SPLIT
    # configs): still behind the split pairs (level 1 chain 40.1 vs 38.1 us, level 2 37.1 vs 28.6;
    # profiles/r05i_dwpw_split_ab.txt)
    DW_FUSE_STRIDES = (8,)

    def fuse_dw(self):
        """Merge each depthwise op D into the 1x1 conv B that immediately follows it and is the only reader of D's
        whole output (the Detect head's cv3.l.0 / cv3.l.1 pairs): B reads D's input and computes act(dw3x3 + bias)
        in registers as its B operand (csrc/ym_conv_dwpw.hip); D's output buffer is never written.  The depthwise
        arithmetic is the unfused op's (same fmaf order, same x3 split), so the 1x1 sees the same operands."""
        out: List[Op] = []
        i = 0
        while i < len(self.ops):
            op = self.ops[i]
            nxt = self.ops[i + 1] if i + 1 < len(self.ops) else None
            if op.kind == "dwconv" and nxt is not None and self._dw_fusable(op, nxt):
                d = op.args
                args = dict(nxt.args)
                args.update(src0=d["src"], dw=dict(wkey=d["wkey"], act=d["act"], C=d["C"]))
                out.append(Op("conv", args, f"{op.name}+{nxt.name.rsplit('.', 1)[-1]}"))
                i += 2
                continue
            out.append(op)
            i += 1
        self.ops = out

    def _dw_fuse_strides(self):
        import os
        e = os.environ.get("YM_DW_FUSE_STRIDES")  # A/B override, e.g. "8,16,32"
        return tuple(int(v) for v in e.split(",") if v) if e else self.DW_FUSE_STRIDES

    def _dw_fusable(self, D: Op, B: Op) -> bool:
        d = D.args
        if B.kind != "conv" or not d["act"] or d["src"].buf.f not in self._dw_fuse_strides():
            return False
        b = B.args
        mid = d["dst"]
        return (b["k"] == 1 and b["s"] == 1 and b["src1"] is None and not b["up0"] and not b["shuffle2x2"]
                and not b.get("convT") and b["res"] is None and b["anchor_level"] < 0 and not b.get("pair")
                and b["src0"].buf is mid.buf and mid.coff == 0 and mid.C == mid.buf.C and b["src0"].C == mid.C
                and self._readers(mid.buf) == 1 and d["C"] % 8 == 0 and d["C"] <= self.DW_MAX_C
                and b["c2"] % 4 == 0 and b["c2"] <= self.DW_MAX_N)

    # csrc/ym_conv_bneck.hip: the (C, C_mid, C_out) Bottleneck shapes with a fused kernel
    BNECK_SHAPES = {(16, 8, 16), (32, 16, 32), (64, 32, 64), (32, 32, 32), (64, 64, 64)}

    def _fusable(self, A: Op, B: Op) -> bool:
        if A.kind != "conv" or B.kind != "conv":
            return False
        a, b = A.args, B.args
        if a.get("pair") or a.get("convT") or a["shuffle2x2"] or a["res"] is not None or a["anchor_level"] >= 0:
            return False
        if a.get("dw") or b.get("dw"):  # a depthwise-fused 1x1 runs on its own kernel (csrc/ym_conv_dwpw.hip)
            return False
        if b["k"] == 3:  # a Bottleneck (3x3 -> 3x3 + shortcut) on the fused kernel of csrc/ym_conv_bneck.hip
            mid = a["dst"]
            return (a["k"] == 3 and a["s"] == 1 and b["s"] == 1 and a["src1"] is None and not a["up0"]
                    and b["src1"] is None and not b["up0"] and not b["shuffle2x2"] and b["anchor_level"] < 0
                    and b["src0"].buf is mid.buf and mid.coff == 0 and mid.C == mid.buf.C
                    and self._readers(mid.buf) == 1  # a Bottleneck: the shortcut is the first conv's input
                    and b["res"] is not None and b["res"].buf is a["src0"].buf and b["res"].coff == a["src0"].coff
                    and b["res"].C == a["src0"].C
                    and (a["c1"], a["c2"], b["c2"]) in self.BNECK_SHAPES)
        if b["k"] != 1 or b["s"] != 1 or b["src1"] is not None or b["up0"] or b["shuffle2x2"] or b.get("convT"):
            return False
        mid = a["dst"]
        if b["src0"].buf is not mid.buf or mid.coff != 0 or mid.C != mid.buf.C or b["src0"].C != mid.C:
            return False
        if self._readers(mid.buf) != 1:
            return False
        if a["k"] == 3 and (a["src1"] is not None or a["up0"]):
            return False
        N, N2 = a["c2"], b["c2"]
        if (self.x3 and a["k"] == 3 and N <= self.DMA_FUSE_MAX and N2 <= self.DMA_FUSE_MAX and N % 8 == 0
                and N2 % 8 == 0 and b["res"] is None):
            return True  # the LDS-DMA kernel's fused-epilogue GEMM (csrc/ym_conv_dma.hip FUSE) takes any K
        xs = 2 if self.x3 else 1  # x3: fp16 storage K of the pair-chunk rows, W2 in hi and lo planes
        kpad = -(-xs * a["k"] * a["k"] * a["c1"] // 64) * 64
        if N > self.FUSE_MAX_N or N % 4 or N2 % 4 or kpad // 32 not in self.STREAM_KS[a["k"]]:
            return False
        if self.x3 and (kpad // 32) % 2:
            return False
        NP, N2P = -(-N // 16) * 16, -(-N2 // 16) * 16
        if NP * (kpad + 16) * 2 + NP * 4 > 80 * 1024:  # csrc/ym_conv_stream.hip LDS: W [NP][Kpad + 16], W2 [N2P][NP + 8]
            return False
        return NP * (kpad + 16) * 2 + NP * 4 + xs * N2P * (NP + 8) * 2 + N2P * 4 <= self.FUSE_MAX_LDS

    # ------------------------------------------------------------------ accounting
    def op_costs(self, B: int, H: int, W: int, act_bytes: int = 2):
        """Per op (aligned with self.ops): (algorithmic FLOPs, algorithmic HBM bytes) for one forward of B images.
        FLOPs = 2·MACs (stem counted at its real Cin=3); bytes = each input element read once + weights +
        outputs written once (+ residual read), at the storage dtype."""
        out = []
        for op in self.ops:
            a = op.args
            fl, by = 0, 0
            if op.kind == "conv":
                fo = self.out_factor(op)
                npx = B * (H // fo) * (W // fo)
                cin = 3 if op.name == "model.0" else a["c1"]
                fl = 2 * npx * a["k"] * a["k"] * cin * a["c2"]
                f0 = a["src0"].buf.f
                by += B * (H // f0) * (W // f0) * a["src0"].C * act_bytes
                if a["src1"] is not None:
                    f1 = a["src1"].buf.f
                    by += B * (H // f1) * (W // f1) * a["src1"].C * act_bytes
                by += a["k"] * a["k"] * cin * a["c2"] * act_bytes + a["c2"] * 4
                if a.get("dw"):  # the fused depthwise: its taps, weights and bias (its output never reaches HBM)
                    fl += 2 * npx * 9 * a["c1"]
                    by += 10 * a["c1"] * 4
                c_out = a["c2"]
                if a.get("pair"):  # + the second conv; its input (this conv's output) never reaches HBM
                    c_out, k2 = a["pair"]["c2"], a["pair"]["k"]
                    fl += 2 * npx * k2 * k2 * a["c2"] * c_out
                    by += k2 * k2 * a["c2"] * c_out * act_bytes + c_out * 4
                ob = 4 if a["dst"].buf.f32 else act_bytes
                by += npx * c_out * ob
                if a["res"] is not None:
                    by += npx * c_out * act_bytes
            elif op.kind == "dwconv":
                f = a["src"].buf.f
                npx = B * (H // f) * (W // f)
                fl = 2 * npx * 9 * a["C"]
                by = 2 * npx * a["C"] * act_bytes
            elif op.kind == "sppf":
                f = a["dst"].f
                npx = B * (H // f) * (W // f)
                by = 4 * npx * a["C"] * act_bytes
            elif op.kind == "attn":
                f = a["qkv"].buf.f
                N = (H // f) * (W // f)
                fl = 2 * B * (N * N * a["nh"] * (a["kd"] + a["hd"]) + N * 9 * a["C"])
                by = B * N * (a["qkv"].C + a["C"]) * act_bytes
            elif op.kind == "requant":
                s_, d_ = a["src"], a["dst"]
                f = d_.buf.f
                npx = B * (H // f) * (W // f)
                by = 2 * npx * d_.C * act_bytes
            elif op.kind == "input":  # LoadTensor statistic: the fp32 NCHW batch read once (the stem reads it again)
                by = B * H * W * 3 * 4
            elif op.kind == "decode":
                A = sum((H // s) * (W // s) for s in STRIDES)
                by = B * A * (a["anchor"].C * 4 + 24)
            out.append((fl, by))
        return out

    def macs_per_image(self, H: int = 640, W: int = 640) -> int:
        # exact count from conv op geometry
        tot = 0
        for op in self.ops:
            a = op.args
            if op.kind == "conv":
                fo = self.out_factor(op)
                npx = (H // fo) * (W // fo)
                tot += npx * a["k"] * a["k"] * (a["c1"] if op.name != "model.0" else 3) * a["c2"]
                if a.get("dw"):
                    tot += npx * 9 * a["c1"]
                if a.get("pair"):
                    tot += npx * a["pair"]["k"] ** 2 * a["c2"] * a["pair"]["c2"]
            elif op.kind == "dwconv":
                f = a["src"].buf.f
                tot += (H // f) * (W // f) * 9 * a["C"]
            elif op.kind == "attn":
                f = a["qkv"].buf.f
                N = (H // f) * (W // f)
                tot += N * N * a["nh"] * (a["kd"] + a["hd"]) + N * 9 * a["C"]
        return tot

    def out_factor(self, op: Op) -> int:
        a = op.args
        fin = a["src0"].buf.f // (2 if a["up0"] else 1)
        if a["anchor_level"] >= 0:
            return fin
        return fin * a["s"]


def _cls_shift(scale: str) -> float:
    from .synth import CLS_BIAS_SHIFT
    return CLS_BIAS_SHIFT[scale]


def infer_arch(sd) -> Tuple[str, str, int]:
    """(scale, task, nc) of an Ultralytics-key state dict: the reference takes the architecture from the checkpoint
    (`YOLO(model_path)`, core/model.py:100-110), so a loaded file decides the plan, not the `size` argument.  The
    task comes from the Proto keys, nc from the last cls conv, the scale from the graph whose every parameter shape
    matches."""
    import numpy as np
    task = "segment" if any(k.startswith("model.23.proto.") for k in sd) else "detect"
    key = "model.23.cv3.0.2.bias"
    if key not in sd:
        raise ValueError(f"not a YOLO11 detect/segment state dict (no {key!r})")
    nc = int(np.shape(sd[key])[0])
    for scale in SCALES:
        g = GraphBuilder(scale, task, nc=nc)
        if all(p.kind in ("count", "dfl") or (p.name in sd and tuple(np.shape(sd[p.name])) == tuple(p.shape))
               for p in g.params):
            return scale, task, nc
    raise ValueError(f"state dict matches no YOLO11 scale ({'/'.join(SCALES)}) for task {task}, nc={nc}")


def param_specs(scale: str = "n", task: str = "detect"):
    g = GraphBuilder(scale, task)
    return [(p.name, p.shape, p.kind, p.extra) for p in g.params]
