"""PTQ int8 restatement of the reference's `PostTrainingQuantizer` on the YOLO11 oracle.  TEST INFRASTRUCTURE ONLY.

Reference: /root/reference/optimization/quantization/quantizers.py
  :42       default backend 'qnnpack'
  :124-131  qconfig = torch.quantization.get_default_qconfig(backend):
              qnnpack: activations HistogramObserver(quint8, per-tensor affine, reduce_range=False) -> [0, 255],
                       weights MinMaxObserver(qint8, per-tensor symmetric)
              fbgemm:  activations HistogramObserver(reduce_range=True) -> [0, 127],
                       weights PerChannelMinMaxObserver(qint8, per-channel symmetric, axis 0)
  :135      torch.quantization.prepare (observers)   :146-177 calibration = forward passes of the float model
  :77       torch.quantization.convert (quantized::conv2d: uint8 activations x int8 weights, int32 accumulation,
            requantisation of the conv output to the output observer's (scale, zero point))
The reference inserts no QuantStub/DeQuantStub and fuses no modules (:93-144), and falls back to the float model on
failure (:217-220), so what it emits is not a stable numeric contract.  This file pins
the build's explicit restatement of that qconfig on the BN-fused YOLO11 graph (AutoBackend fuses before predict):

  * every Conv2d / ConvTranspose2d (incl. depthwise, Attention.pe, the Detect/Segment head convs) is a quantized
    conv: acc = sum (q_x - z_x) * q_w (exact int32), y = float(acc) * (s_x * s_w) + bias (fp32, two roundings),
    q_out = clamp(round_half_even(y * (1 / s_out)) + z_out, qmin, qmax) with (s_out, z_out) = the conv's output
    observer ("out:<module path>");
  * SiLU, residual adds, concats, the attention matmuls and softmax, the DFL decode run in float between the
    quantized convs: the conv output is dequantised ((q - z) * s), activated (SiLU evaluated in float64, rounded
    once to fp32), and quantized again with the observer of the TENSOR it is stored in ("act:<tensor name>");
  * a tensor has ONE observer: a concat's members are quantized with the concat's, a chunk/split view inherits its
    parent's (the QuantStub sits after the producer, not in front of each consumer, so int8 storage stays
    zero-copy);
  * act=False convs stored as they are (Attention.qkv, Proto.upsample) keep their output quantisation as the stored
    tensor's; terminal head outputs (Detect box/cls, Segment coefficients, Proto.cv3) are dequantised to float;
  * max-pool and nearest upsample act on the quantized values; DFL's fixed arange projection is part of the float
    decode; ConvTranspose2d weights are per-tensor on both backends;
  * the attention core (q·kᵀ·scale, softmax, ·v, on the dequantised fp32 q/k/v) is evaluated in float64 and rounded
    to fp32 once, at its output: an order-independent float island, so the int8 model is bit-reproducible across
    implementations (fp32 accumulation would make one rounding flip cascade through the later int8 layers);
  * the weights quantized are the BN-fused fp32 weights of an elementwise fold (W * (g / sqrt(eps + var)),
    b' = beta - (g * mean) / sqrt(var + eps), eps 1e-3, IEEE-rounded sqrt): `fuse_conv_and_bn` without its
    diag-matrix BLAS product.
Tensor names are Ultralytics module paths (act:model.2.cat, act:model.12 = layer 12's Concat, out:model.2.cv1).
Agreement with torch.ao's own quantized kernels is checked in tests/test_quant_oracle.py (quantized::conv2d).

Backend "fp8" is the fp8 variant BASELINE config 4 names ("PTQ int8 ... fp8 MFMA"; SURVEY §8(c): e4m3 emulated by
torch.float8_e4m3fn casts): the same quantisation points and structure, with every quantized tensor an OCP e4m3
value (the gfx950 fp8 format) times a per-tensor scale s = amax / 448 from a min/max observer (zero point 0), code
= e4m3(clamp(v * (1/s), +-448)) rounded to nearest even; weights e4m3 per output channel (s[n] = max|w[n]| / 448).
A QT then holds the decoded e4m3 values in `q` (z = 0), so (q - z) * s is the dequantised tensor exactly as for
int8, and a conv's float64 accumulation of e4m3 products is exact (8-bit significands).  accum="mfma" replaces that
exact sum, for every dense conv the GPU plan runs on the fp8 MFMA, by the instruction's own accumulation restated
(mfma_f8_step, fitted to the hardware's outputs; mfma_f8_conv, in the GPU kernel's K order): the oracle the fp8 plan
is bit-exact against, layer by layer (tests/test_gpu_fp8.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.ao.quantization.observer import HistogramObserver, MinMaxObserver, PerChannelMinMaxObserver

from . import postprocess as pp
from .yolo11 import C3k, Conv, YOLO11, build

# backend -> (activation reduce_range, per-channel w)
BACKENDS = {"qnnpack": (False, False), "fbgemm": (True, True), "fp8": (False, True)}
F32 = np.float32
E4M3_MAX = 448.0


def silu64(x: torch.Tensor) -> torch.Tensor:
    """SiLU of fp32 values evaluated in float64 and rounded once to fp32 (machine-independent tables)."""
    d = x.double()
    return (d / (1.0 + torch.exp(-d))).float()


def _t32(v: float) -> torch.Tensor:
    return torch.tensor(F32(v), dtype=torch.float32)


def inv32(s: float) -> float:
    return float(F32(1.0) / F32(s))


class QT:
    """A stored quantized tensor: integer values q (float32 holding exact ints), scale s (an fp32 value), zp z."""

    __slots__ = ("q", "s", "z")

    def __init__(self, q: torch.Tensor, s: float, z: int):
        self.q, self.s, self.z = q, float(F32(s)), int(z)

    def deq(self) -> torch.Tensor:
        return (self.q - self.z) * _t32(self.s)

    def slice(self, a: int, b: int) -> "QT":
        return QT(self.q[:, a:b], self.s, self.z)


def quantize(v: torch.Tensor, s: float, z: int, qmin: int, qmax: int) -> torch.Tensor:
    return torch.clamp(torch.round(v * _t32(inv32(s))) + z, qmin, qmax)


# --------------------------------------------------------------------------------------------------------------------
# The gfx950 fp8 MFMA, restated (round 6).  tools/f8_mfma_probe.hip fed known e4m3 operands to
# v_mfma_f32_32x32x16_fp8_fp8 (profiles/r05h_f8_mfma_probe.txt); tools/f8_mfma_model.py then found the accumulation
# (profiles/r06_f8_mfma_model.txt; 524,288 outputs, 99.997 % bit-exact, the rest within 2 fp32 ulps):
#   * the 16 products of one output form two groups of 8 — the 8 consecutive k of each lane half;
#   * in a group every product a·b (exact: 4-bit x 4-bit significands) is aligned to the group's largest exponent
#     sum E_g = max(e_a + e_b) over its nonzero products (e = the unbiased exponent, -6 for subnormals), truncated
#     toward zero to a multiple of 2^(E_g - 13), and the 8 are summed exactly;
#   * the two group sums and C are aligned to E = max(E_g0 + 1, E_g1 + 1, exponent of C), floored to a multiple of
#     2^(E - 25), summed exactly, and that sum is rounded once to fp32 (nearest even).
# Round 5 had compared the instruction with fl32(C + exact sum) only (24 % equal) and fitted truncations relative to
# the whole K, which do not fit; the per-group exponent sums do.  tests/golden/f8_mfma_probe.npz holds a sample of the
# probe's operands and the hardware's outputs (tests/test_fp8_oracle.py checks mfma_f8_step against them).
_NEG = -(1 << 20)


def e4m3_parts(v: torch.Tensor):
    """(signed significand, exponent) int32 tensors of e4m3 VALUES v (v = sig * 2^(e - 3); subnormals e = -6)."""
    code = v.float().to(torch.float8_e4m3fn).view(torch.uint8).to(torch.int32)
    f, m = (code >> 3) & 15, code & 7
    sig = torch.where(f == 0, m, m + 8)
    e = torch.where(f == 0, torch.full_like(f, -6), f - 7)
    return torch.where((code & 0x80) != 0, -sig, sig), e


def mfma_f8_step(C: torch.Tensor, sa, ea, sb, eb) -> torch.Tensor:
    """One v_mfma_f32_32x32x16_fp8_fp8 accumulation per output, restated above.  C (...) fp32; sa/ea and sb/eb
    broadcastable (..., 2, 8) int32: significands / exponents of the two 8-product groups of each output."""
    mp = sa * sb
    es = ea + eb
    nz = mp != 0
    Eg = torch.where(nz, es, torch.full_like(es, _NEG)).amax(-1)  # (..., 2)
    d = Eg.unsqueeze(-1) - es
    mag = mp.abs()
    q = torch.where(d <= 7, mag << (7 - d).clamp(0, 7), mag >> (d - 7).clamp(0, 30))  # units 2^(E_g - 13)
    S = torch.where(nz, torch.where(mp < 0, -q, q), torch.zeros_like(q)).sum(-1).to(torch.int64)
    man, ex = torch.frexp(C.double())
    cz = C == 0
    ec = torch.where(cz, torch.full_like(ex, _NEG), ex - 1).to(torch.int64)
    mc = torch.where(cz, torch.zeros_like(man), man * 2.0 ** 24).to(torch.int64)  # C = mc * 2^(ec - 23)
    gv = Eg > _NEG // 2
    E = torch.maximum(torch.where(gv, Eg + 1, torch.full_like(Eg, _NEG)).amax(-1).to(torch.int64), ec)
    kg = Eg.to(torch.int64) - E.unsqueeze(-1) + 12
    tg = torch.where(kg >= 0, S << kg.clamp(0, 40), S >> (-kg).clamp(0, 62))  # floor
    kc = ec - E + 2
    tc = torch.where(kc >= 0, mc << kc.clamp(0, 40), mc >> (-kc).clamp(0, 62))
    T = torch.where(gv, tg, torch.zeros_like(tg)).sum(-1) + torch.where(cz, torch.zeros_like(tc), tc)
    out = (T.double() * torch.pow(2.0, E.double() - 25)).float()
    return torch.where(E > _NEG // 2, out, torch.zeros_like(out))


def mfma_f8_conv(xv: torch.Tensor, wv: torch.Tensor, stride, padding) -> torch.Tensor:
    """conv2d of e4m3 values xv (B, C, H, W) and wv (N, C, k, k) as the GPU fp8 plan's conv_i8 kernel accumulates it
    (csrc/ym_conv_i8.hip, one K chain per output): K ordered (ky, kx, c) and zero-padded to a multiple of 64, each
    32-deep step t two fp8 MFMAs — the first over K = 32t + 16h + j, the second over 32t + 16h + 8 + j (lane half h,
    j < 8: bytes 0-7 and 8-15 of the lane's 16-byte chunk) — chained through C from 0.  Returns fp32 (B, N, Ho, Wo)."""
    B, Cin, H, W = xv.shape
    N, _, kh, kw = wv.shape
    s = stride[0] if isinstance(stride, (tuple, list)) else stride
    p = padding[0] if isinstance(padding, (tuple, list)) else padding
    Ho, Wo = (H + 2 * p - kh) // s + 1, (W + 2 * p - kw) // s + 1
    K = kh * kw * Cin
    Kp = -(-K // 64) * 64
    cols = F.unfold(xv.float(), (kh, kw), padding=p, stride=s)  # (B, C*k*k, L), index c*k*k + tap
    cols = cols.view(B, Cin, kh * kw, Ho * Wo).permute(0, 3, 2, 1).reshape(B * Ho * Wo, K)
    wm = wv.float().permute(0, 2, 3, 1).reshape(N, K)
    if Kp > K:
        cols = F.pad(cols, (0, Kp - K))
        wm = F.pad(wm, (0, Kp - K))
    T = Kp // 32
    xs, xe = (t.view(-1, T, 2, 2, 8) for t in e4m3_parts(cols))  # (M, t, h, u, j)
    ws, we = (t.view(N, T, 2, 2, 8) for t in e4m3_parts(wm))
    M = cols.shape[0]
    out = torch.empty((M, N), dtype=torch.float32)
    mc = max(1, (1 << 21) // N)
    for m0 in range(0, M, mc):
        m1 = min(M, m0 + mc)
        acc = torch.zeros((m1 - m0, N), dtype=torch.float32)
        for t in range(T):
            for u in range(2):
                acc = mfma_f8_step(acc, xs[m0:m1, t, :, u, None, :].transpose(1, 2), xe[m0:m1, t, :, u, None, :].transpose(1, 2),
                                   ws[None, :, t, :, u, :], we[None, :, t, :, u, :])
        out[m0:m1] = acc
    return out.view(B, Ho, Wo, N).permute(0, 3, 1, 2).contiguous()


def fp8_scale(amax: float) -> float:
    """e4m3 scale of an observed range: amax / 448 in fp32 (1 / 448 for an all-zero tensor)."""
    amax = float(amax)
    return float(F32(amax) / F32(E4M3_MAX)) if amax > 0 else float(F32(1.0) / F32(E4M3_MAX))


def quantize_fp8(v: torch.Tensor, s: float) -> torch.Tensor:
    """e4m3 VALUES (as fp32) of v * (1/s): clamp to +-448, then torch's round-to-nearest-even float8_e4m3fn cast."""
    return torch.clamp(v.float() * _t32(inv32(s)), -E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float()


def quantize_weight_fp8(w: torch.Tensor) -> Tuple[torch.Tensor, np.ndarray]:
    """Per-output-channel e4m3 weights over axis 0: (e4m3 values as fp32, fp32 scale per channel)."""
    w = w.detach().float().contiguous()
    amax = w.abs().reshape(w.shape[0], -1).amax(1)
    s = np.array([fp8_scale(float(a)) for a in amax], F32)
    inv = torch.from_numpy((F32(1.0) / s).astype(F32)).view(-1, *([1] * (w.dim() - 1)))
    return torch.clamp(w * inv, -E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float(), s


def quantize_weight(w: torch.Tensor, per_channel: bool) -> Tuple[torch.Tensor, np.ndarray]:
    """torch.ao weight observer + quantize: (int8 values as float32, per-output-channel fp32 scales)."""
    w = w.detach().float().contiguous()
    if per_channel:
        obs = PerChannelMinMaxObserver(ch_axis=0, dtype=torch.qint8, qscheme=torch.per_channel_symmetric)
        obs(w)
        s, z = obs.calculate_qparams()
        wq = torch.quantize_per_channel(w, s.double(), z.long(), 0, torch.qint8).int_repr().float()
        return wq, s.float().numpy().astype(F32)
    obs = MinMaxObserver(dtype=torch.qint8, qscheme=torch.per_tensor_symmetric)
    obs(w)
    s, _ = obs.calculate_qparams()
    wq = torch.quantize_per_tensor(w, float(s), 0, torch.qint8).int_repr().float()
    return wq, np.full(w.shape[0], F32(float(s)), F32)


def _sqrt32(t: torch.Tensor) -> torch.Tensor:
    """Correctly rounded fp32 sqrt (torch's vectorised CPU sqrt is not always; IEEE sqrt in float64 then one
    rounding is)."""
    return torch.sqrt(t.double()).float()


def fold_elementwise(net: YOLO11) -> YOLO11:
    """Fold every Conv's BN into its conv with the elementwise fp32 formula (see the module docstring)."""
    for m in net.modules():
        if isinstance(m, Conv) and not m.fused:
            conv, bn = m.conv, m.bn
            eps = _t32(bn.eps)
            g, beta = bn.weight.detach().float(), bn.bias.detach().float()
            mean, var = bn.running_mean.detach().float(), bn.running_var.detach().float()
            scale = g / _sqrt32(eps + var)
            fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                              groups=conv.groups, bias=True).requires_grad_(False)
            fused.weight.copy_(scale.view(-1, 1, 1, 1) * conv.weight.detach().float())
            fused.bias.copy_(beta - (g * mean) / _sqrt32(var + eps))
            m.conv = fused
            del m.bn
            m.fused = True
    return net


class _Ctx:
    """One walk over the fused oracle graph: mode 'float' (plain fp32), 'observe' (fp32 + observers, calibration) or
    'quant' (int8 arithmetic with the calibrated qparams)."""

    def __init__(self, backend: str, mode: str, qparams: Optional[Dict] = None, accum: str = "exact"):
        if backend not in BACKENDS:
            raise ValueError(f"backend {backend!r} not in {list(BACKENDS)}")
        if accum not in ("exact", "mfma") or (accum == "mfma" and backend != "fp8"):
            raise ValueError(f"accum {accum!r}: 'exact', or 'mfma' for the fp8 backend")
        self.backend, self.mode = backend, mode
        self.fp8 = backend == "fp8"
        # fp8 convs: "exact" = float64 sums rounded once; "mfma" = the fp8 MFMA chain of the GPU plan (mfma_f8_conv) for
        # every dense conv with more than 3 input channels (the stem and the depthwise convs stay exact on the GPU too)
        self.accum = accum
        self.reduce_range, self.per_channel = BACKENDS[backend]
        self.qmin, self.qmax = 0, (127 if self.reduce_range else 255)
        self.obs: Dict[str, HistogramObserver] = {}
        self.qp = qparams or {}
        self.wcache: Dict[str, tuple] = {}
        self.trace: Optional[Dict[str, "QT"]] = None  # quant mode: every stored tensor by quantisation key

    @property
    def quant(self) -> bool:
        return self.mode == "quant"

    def _observe(self, key: str, t: torch.Tensor):
        if self.mode != "observe":
            return
        o = self.obs.get(key)
        if o is None:
            o = self.obs[key] = (MinMaxObserver(dtype=torch.quint8, qscheme=torch.per_tensor_affine) if self.fp8 else
                                 HistogramObserver(dtype=torch.quint8, qscheme=torch.per_tensor_affine,
                                                   reduce_range=self.reduce_range))
        o(t.detach().float())

    def _quantize(self, v: torch.Tensor, s: float, z: int) -> torch.Tensor:
        return quantize_fp8(v, s) if self.fp8 else quantize(v, s, z, self.qmin, self.qmax)

    # ---- tensors
    def store(self, name: str, v: torch.Tensor):
        """A float tensor becomes a stored tensor (quantized with act:<name>)."""
        self._observe("act:" + name, v)
        q = self.qwith(name, v)
        if self.trace is not None and self.quant:
            self.trace["act:" + name] = q
        return q

    def qwith(self, name: str, v: torch.Tensor):
        """Quantize with act:<name> without observing (a member of a concat observed as a whole)."""
        if not self.quant:
            return v
        s, z = self.qp["act:" + name]
        return QT(self._quantize(v, s, z), s, z)

    def cat(self, name: str, parts: List):
        if not self.quant:
            c = torch.cat(parts, 1)
            self._observe("act:" + name, c)
            return c
        c = QT(torch.cat([p.q for p in parts], 1), parts[0].s, parts[0].z)
        if self.trace is not None:
            self.trace["act:" + name] = c
        return c

    def deq(self, x):
        return x.deq() if self.quant else x

    def slice(self, x, a: int, b: int):
        return x.slice(a, b) if self.quant else x[:, a:b]

    def add(self, v: torch.Tensor, x):
        return v + self.deq(x)

    def pool(self, m: nn.MaxPool2d, x):
        return QT(m(x.q), x.s, x.z) if self.quant else m(x)

    # ---- convs
    def weights(self, name: str, mod: nn.Module):
        if name not in self.wcache:
            convT = isinstance(mod, nn.ConvTranspose2d)
            if self.fp8:
                if convT:
                    raise ValueError("the fp8 plan covers detect models (no ConvTranspose2d)")
                self.wcache[name] = quantize_weight_fp8(mod.weight)
                return self.wcache[name]
            wq, sw = quantize_weight(mod.weight, self.per_channel and not convT)
            if convT:  # (in, out, kh, kw): one per-tensor scale, broadcast over the output channels
                sw = np.full(mod.weight.shape[1], sw[0], F32)
            self.wcache[name] = (wq, sw)
        return self.wcache[name]

    def conv(self, name: str, mod: nn.Module, x, act: bool):
        """Quantized conv (mod: fused nn.Conv2d with bias, or nn.ConvTranspose2d). Returns (post, stored): post =
        the float activation of the (requantised) output, stored = the output as a tensor in its own quantisation."""
        if not self.quant:
            y = mod(x)
            self._observe("out:" + name, y)
            post = F.silu(y) if act else y
            return post, post
        wq, sw = self.weights(name, mod)
        xi = (x.q - x.z).double()
        if isinstance(mod, nn.ConvTranspose2d):
            acc = F.conv_transpose2d(xi, wq.double(), None, mod.stride, mod.padding)
        elif self.accum == "mfma" and mod.groups == 1 and mod.in_channels > 3:
            acc = mfma_f8_conv(x.q, wq, mod.stride, mod.padding)  # (fp8: z = 0, so x.q - x.z = x.q)
        else:
            acc = F.conv2d(xi, wq.double(), None, mod.stride, mod.padding, mod.dilation, mod.groups)
        sasw = _t32(x.s) * torch.from_numpy(sw)  # fp32 product per output channel
        y = acc.float() * sasw.view(1, -1, 1, 1)
        y = y + mod.bias.detach().float().view(1, -1, 1, 1)
        so, zo = self.qp["out:" + name]
        stored = QT(self._quantize(y, so, zo), so, zo)
        if self.trace is not None:
            self.trace["out:" + name] = stored
            self.trace["y:" + name] = y
        deq = stored.deq()
        return (silu64(deq) if act else deq), stored


def _cv(ctx: _Ctx, name: str, c, x):
    """Ultralytics `Conv` (fused): returns the float post-activation."""
    return ctx.conv(name, c.conv, x, not isinstance(c.act, nn.Identity))[0]


def _bottleneck(ctx, p, m, x):
    h = ctx.store(p + ".cv1", _cv(ctx, p + ".cv1", m.cv1, x))
    v = _cv(ctx, p + ".cv2", m.cv2, h)
    return ctx.add(v, x) if m.add else v


def _c3k(ctx, p, m, x):
    cur = ctx.store(p + ".cv1", _cv(ctx, p + ".cv1", m.cv1, x))
    mods = list(m.m)
    last = None
    for j, b in enumerate(mods):
        v = _bottleneck(ctx, f"{p}.m.{j}", b, cur)
        if j < len(mods) - 1:
            cur = ctx.store(f"{p}.m.{j}", v)
        else:
            last = v
    v2 = _cv(ctx, p + ".cv2", m.cv2, x)
    catn = p + ".cat"
    cat = ctx.cat(catn, [ctx.qwith(catn, last), ctx.qwith(catn, v2)])
    return _cv(ctx, p + ".cv3", m.cv3, cat)


def _c3k2(ctx, i, m, x):
    """C3k2 / C2f: y = cv1(x).chunk(2); y += [m_j(y[-1])]; cv2(cat(y))."""
    p = f"model.{i}"
    catn = p + ".cat"
    c = m.c
    parts = [ctx.qwith(catn, _cv(ctx, p + ".cv1", m.cv1, x))]
    last = ctx.slice(parts[0], c, 2 * c)
    for j, mm in enumerate(m.m):
        pj = f"{p}.m.{j}"
        v = _c3k(ctx, pj, mm, last) if isinstance(mm, C3k) else _bottleneck(ctx, pj, mm, last)
        parts.append(ctx.qwith(catn, v))
        last = parts[-1]
    cat = ctx.cat(catn, parts)
    return ctx.store(p, _cv(ctx, p + ".cv2", m.cv2, cat))


def _sppf(ctx, i, m, x):
    p = f"model.{i}"
    catn = p + ".cat"
    ys = [ctx.qwith(catn, _cv(ctx, p + ".cv1", m.cv1, x))]
    for _ in range(3):
        ys.append(ctx.pool(m.m, ys[-1]))
    cat = ctx.cat(catn, ys)
    return ctx.store(p, _cv(ctx, p + ".cv2", m.cv2, cat))


def _psablock(ctx, p, blk, b):
    at = blk.attn
    bf = ctx.deq(b)
    B, C, H, W = bf.shape
    N = H * W
    nh, kd, hd = at.num_heads, at.key_dim, at.head_dim
    _, qkv = ctx.conv(p + ".attn.qkv", at.qkv.conv, b, False)  # stored as is (its own output quantisation)
    qkvf = ctx.deq(qkv)
    q, k, v = qkvf.view(B, nh, 2 * kd + hd, N).split([kd, kd, hd], dim=2)
    if ctx.quant:  # the float island of the int8 model, evaluated in float64 and rounded once (see module docstring)
        s64 = (q.double().transpose(-2, -1) @ k.double()) * float(F32(at.scale))
        o = (v.double() @ s64.softmax(dim=-1).transpose(-2, -1)).float().view(B, C, H, W)
    else:
        attn = ((q.transpose(-2, -1) @ k) * at.scale).softmax(dim=-1)
        o = (v @ attn.transpose(-2, -1)).view(B, C, H, W)
    if ctx.quant:
        vq = QT(qkv.q.view(B, nh, 2 * kd + hd, N)[:, :, 2 * kd:, :].reshape(B, C, H, W), qkv.s, qkv.z)
    else:
        vq = v.reshape(B, C, H, W)
    pe = _cv(ctx, p + ".attn.pe", at.pe, vq)
    xo = ctx.store(p + ".attn.x", o + pe)
    b1 = ctx.store(p + ".attn_add", ctx.add(_cv(ctx, p + ".attn.proj", at.proj, xo), b))
    f0 = ctx.store(p + ".ffn.0", _cv(ctx, p + ".ffn.0", blk.ffn[0], b1))
    return ctx.store(p, ctx.add(_cv(ctx, p + ".ffn.1", blk.ffn[1], f0), b1))


def _c2psa(ctx, i, m, x):
    p = f"model.{i}"
    t = ctx.store(p + ".cv1", _cv(ctx, p + ".cv1", m.cv1, x))
    a, b = ctx.slice(t, 0, m.c), ctx.slice(t, m.c, 2 * m.c)
    for j, blk in enumerate(m.m):
        b = _psablock(ctx, f"{p}.m.{j}", blk, b)
    cat = ctx.store(p + ".cat", torch.cat([ctx.deq(a), ctx.deq(b)], 1))
    return ctx.store(p, _cv(ctx, p + ".cv2", m.cv2, cat))


def _up(t: torch.Tensor) -> torch.Tensor:
    return F.interpolate(t, scale_factor=2.0, mode="nearest")


def _head(ctx, m, xs, task):
    p = "model.23"
    extra = {}
    if task == "segment":
        pr = m.proto
        p1 = ctx.store(p + ".proto.cv1", _cv(ctx, p + ".proto.cv1", pr.cv1, xs[0]))
        _, p2 = ctx.conv(p + ".proto.upsample", pr.upsample, p1, False)  # stored as is
        p3 = ctx.store(p + ".proto.cv2", _cv(ctx, p + ".proto.cv2", pr.cv2, p2))
        extra["proto"] = _cv(ctx, p + ".proto.cv3", pr.cv3, p3)  # terminal: float
        mcs = []
        for l in range(m.nl):
            s4 = m.cv4[l]
            t1 = ctx.store(f"{p}.cv4.{l}.0", _cv(ctx, f"{p}.cv4.{l}.0", s4[0], xs[l]))
            t2 = ctx.store(f"{p}.cv4.{l}.1", _cv(ctx, f"{p}.cv4.{l}.1", s4[1], t1))
            mc = ctx.conv(f"{p}.cv4.{l}.2", s4[2], t2, False)[0]
            mcs.append(mc.reshape(mc.shape[0], m.nm, -1))
        extra["mc"] = torch.cat(mcs, 2)
    feats = []
    for l in range(m.nl):
        s2, s3 = m.cv2[l], m.cv3[l]
        t1 = ctx.store(f"{p}.cv2.{l}.0", _cv(ctx, f"{p}.cv2.{l}.0", s2[0], xs[l]))
        t2 = ctx.store(f"{p}.cv2.{l}.1", _cv(ctx, f"{p}.cv2.{l}.1", s2[1], t1))
        box = ctx.conv(f"{p}.cv2.{l}.2", s2[2], t2, False)[0]
        d1 = ctx.store(f"{p}.cv3.{l}.0.0", _cv(ctx, f"{p}.cv3.{l}.0.0", s3[0][0], xs[l]))
        e1 = ctx.store(f"{p}.cv3.{l}.0.1", _cv(ctx, f"{p}.cv3.{l}.0.1", s3[0][1], d1))
        d2 = ctx.store(f"{p}.cv3.{l}.1.0", _cv(ctx, f"{p}.cv3.{l}.1.0", s3[1][0], e1))
        e2 = ctx.store(f"{p}.cv3.{l}.1.1", _cv(ctx, f"{p}.cv3.{l}.1.1", s3[1][1], d2))
        cls = ctx.conv(f"{p}.cv3.{l}.2", s3[2], e2, False)[0]
        feats.append(torch.cat((box, cls), 1))
    y = m._inference(feats)
    if task == "segment":
        y = torch.cat([y, extra["mc"]], 1)
    return y, feats, extra


def forward(ctx: _Ctx, net: YOLO11, im: torch.Tensor):
    """The fused YOLO11 forward with quantisation points (SURVEY Appendix A layer order).  im: preprocessed (B,3,H,W)
    fp32.  Returns (y (B, 84[+32], A), feats, extras)."""
    L = net.model
    st = {}
    x = ctx.store("input", im)

    def conv_layer(i, src):
        return ctx.store(f"model.{i}", _cv(ctx, f"model.{i}", L[i], src))

    st[0] = conv_layer(0, x)
    st[1] = conv_layer(1, st[0])
    st[2] = _c3k2(ctx, 2, L[2], st[1])
    st[3] = conv_layer(3, st[2])
    st[4] = _c3k2(ctx, 4, L[4], st[3])
    st[5] = conv_layer(5, st[4])
    st[6] = _c3k2(ctx, 6, L[6], st[5])
    st[7] = conv_layer(7, st[6])
    st[8] = _c3k2(ctx, 8, L[8], st[7])
    st[9] = _sppf(ctx, 9, L[9], st[8])
    st[10] = _c2psa(ctx, 10, L[10], st[9])
    cat12 = ctx.store("model.12", torch.cat([_up(ctx.deq(st[10])), ctx.deq(st[6])], 1))
    st[13] = _c3k2(ctx, 13, L[13], cat12)
    cat15 = ctx.store("model.15", torch.cat([_up(ctx.deq(st[13])), ctx.deq(st[4])], 1))
    st[16] = _c3k2(ctx, 16, L[16], cat15)
    st[17] = conv_layer(17, st[16])
    cat18 = ctx.store("model.18", torch.cat([ctx.deq(st[17]), ctx.deq(st[13])], 1))
    st[19] = _c3k2(ctx, 19, L[19], cat18)
    st[20] = conv_layer(20, st[19])
    cat21 = ctx.store("model.21", torch.cat([ctx.deq(st[20]), ctx.deq(st[10])], 1))
    st[22] = _c3k2(ctx, 22, L[22], cat21)
    y, feats, extra = _head(ctx, L[23], [st[16], st[19], st[22]], net.task)
    extra["stored"] = st
    return y, feats, extra


def build_folded(scale: str, task: str, state_dict: Dict) -> YOLO11:
    return fold_elementwise(build(scale, task, state_dict, fuse=False))


@torch.no_grad()
def calibrate(net: YOLO11, batches: Sequence[torch.Tensor], backend: str = "qnnpack") -> Dict:
    """PostTrainingQuantizer._calibrate_model restated (quantizers.py:146-177): float forwards with observers on every
    conv output and every stored tensor; returns {"backend", "<kind>:<name>": (scale fp32, zero point)}."""
    ctx = _Ctx(backend, "observe")
    for im in batches:
        forward(ctx, net, pp.load_tensor_check(im.float()).float())
    qp = {"backend": backend}
    for k, o in ctx.obs.items():
        if backend == "fp8":
            qp[k] = (fp8_scale(max(abs(float(o.min_val)), abs(float(o.max_val)))), 0)
            continue
        s, z = o.calculate_qparams()
        qp[k] = (float(F32(float(s))), int(z))
    return qp


def qparams_to_json(qp: Dict) -> Dict:
    return {k: (v if k == "backend" else [float(v[0]), int(v[1])]) for k, v in qp.items()}


def qparams_from_json(d: Dict) -> Dict:
    return {k: (v if k == "backend" else (float(F32(v[0])), int(v[1]))) for k, v in d.items()}


class Int8OracleModel:
    """The int8 model's predict (LoadTensor → quantized forward → float decode → NMS → scale_boxes)."""

    def __init__(self, scale: str, task: str, state_dict: Dict, qparams: Dict, accum: str = "exact"):
        self.scale, self.task = scale, task
        self.net = build_folded(scale, task, state_dict)
        self.qp = qparams
        self.ctx = _Ctx(qparams["backend"], "quant", qparams, accum)

    @torch.no_grad()
    def raw(self, im: torch.Tensor):
        im = pp.load_tensor_check(im.float().cpu()).float()
        y, feats, extra = forward(self.ctx, self.net, im)
        return im, y, dict(feats=feats, **extra)

    @torch.no_grad()
    def predict(self, im: torch.Tensor, conf: float = 0.25, iou: float = 0.7, classes=None, agnostic_nms=False,
                max_det: int = 300) -> List[Dict]:
        im, y, ex = self.raw(im)
        nc = 80 if self.task == "segment" else 0
        dets = pp.non_max_suppression(y, conf, iou, classes, agnostic_nms, max_det, nc=nc)
        shape = im.shape[2:]
        out = []
        for d in dets:
            d = d.clone()
            d[:, :4] = pp.scale_boxes(shape, d[:, :4], shape)
            out.append({"boxes": d[:, :6]})
        return out


@torch.no_grad()
def float_walk(net: YOLO11, im: torch.Tensor):
    """The walk in 'float' mode (no quantisation): must reproduce the oracle's own forward."""
    return forward(_Ctx("qnnpack", "float"), net, im)
