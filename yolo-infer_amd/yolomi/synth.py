"""Portable seeded synthetic weights for YOLO11 graphs.

There are no real checkpoints offline (`core/model.py:106-110` of the reference fetches `yolo11{size}.pt` by
name), so every run uses weights synthesised here.  The generator is splitmix64 → uniform → Box-Muller in plain
numpy uint64 arithmetic, so the same (seed, parameter name) gives bit-identical fp32 values on any host and with
any torch version.  Each tensor gets its own stream keyed by FNV-1a(name) ^ seed, so the values do not depend on
the order parameters are enumerated in.

Output is an Ultralytics-style state dict (`model.{i}.conv.weight`, `model.{i}.bn.running_var`, ...) as numpy
fp32 arrays — the same key space a real `yolo11n.pt` state dict uses, so the packer (`yolomi.plan`) works on
either.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Tuple

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of the splitmix64 sequence started at `seed` (vectorised; wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int) -> np.ndarray:
    """U[0,1) float64 from the top 53 bits."""
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, n: int) -> np.ndarray:
    """Standard normal float64 by Box-Muller on pairs of uniforms."""
    m = (n + 1) // 2
    u = uniform(seed, 2 * m)
    u1 = np.maximum(u[0::2], 1e-300)
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * math.pi * u2), r * np.sin(2 * math.pi * u2)])
    return z[:n]


# Tuned once per model family so that synthetic weights give a non-degenerate detector: activations stay O(1)
# through the whole graph and roughly 20-60 anchors per image clear conf=0.25 on U[0,1) images.
CLS_BIAS_SHIFT = {"n": 6.0, "s": 6.0, "m": 6.0, "l": 6.0, "x": 6.0}
CONV_GAIN = 1.6


def synth_param(name: str, shape: Tuple[int, ...], kind: str, seed: int, extra: dict) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    key = fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
    if kind == "conv_w":  # He-normal with a SiLU-ish gain on the true fan-in
        fan_in = int(np.prod(shape[1:]))
        w = normal(key, n) * (CONV_GAIN / math.sqrt(fan_in))
    elif kind == "head_w":  # final 1x1 prediction convs: small
        fan_in = int(np.prod(shape[1:]))
        w = normal(key, n) * (1.0 / math.sqrt(fan_in))
    elif kind == "convT_w":  # ConvTranspose2d weight (in, out, kh, kw): fan-in = in
        w = normal(key, n) * (CONV_GAIN / math.sqrt(shape[0]))
    elif kind == "bn_w":
        w = 1.0 + 0.2 * (uniform(key, n) - 0.5)
    elif kind == "bn_b":
        w = 0.1 * normal(key, n)
    elif kind == "bn_mean":
        w = 0.1 * normal(key, n)
    elif kind == "bn_var":
        w = 0.75 + 0.5 * uniform(key, n)
    elif kind == "box_b":  # Ultralytics Detect.bias_init: box bias 1.0
        w = np.ones(n)
    elif kind == "cls_b":  # Ultralytics bias_init log(5/nc/(640/s)^2), shifted so synthetic images give detections
        nc, stride = extra["nc"], extra["stride"]
        w = np.full(n, math.log(5.0 / nc / (640.0 / stride) ** 2) + extra["shift"])
        w = w + 0.5 * normal(key, n)
    elif kind == "bias":
        w = 0.1 * normal(key, n)
    elif kind == "dfl":  # DFL conv weight is arange(reg_max), not trainable
        w = np.arange(n, dtype=np.float64)
    elif kind == "count":
        return np.zeros(shape, dtype=np.int64)
    else:
        raise ValueError(kind)
    return w.astype(np.float32).reshape(shape)


def synth_state_dict(param_specs: Iterable[Tuple[str, Tuple[int, ...], str, dict]], seed: int = 0
                     ) -> Dict[str, np.ndarray]:
    return {name: synth_param(name, tuple(shape), kind, seed, extra) for name, shape, kind, extra in param_specs}


# ---------------------------------------------------------------------------------------------------------------
# BN running-stat calibration by per-channel moment propagation over the plan (no images, numpy only).
#
# Real checkpoints carry BN running stats measured on data.  Random conv weights with arbitrary BN stats blow up
# through the residual/SPPF/PSA stages (activations of O(100) by the neck, every anchor saturated), so the
# synthesiser sets running_mean/var to the moments each conv's pre-BN output would have if every channel were an
# independent random variable with the moments propagated from a U[0,1) input.  Each BN then emits ≈N(β, γ²).

_GH_X, _GH_W = np.polynomial.hermite.hermgauss(48)


def _silu_moments(mu: np.ndarray, var: np.ndarray):
    s = np.sqrt(np.maximum(var, 1e-12))
    x = mu[:, None] + math.sqrt(2.0) * s[:, None] * _GH_X[None, :]
    f = x / (1.0 + np.exp(-x))
    w = _GH_W[None, :] / math.sqrt(math.pi)
    m1 = (f * w).sum(1)
    m2 = (f * f * w).sum(1)
    return m1, np.maximum(m2 - m1 * m1, 1e-12)


# E[max] and Var[max] of n iid N(0,1) for the SPPF windows (n = 25, 81, 169), by quadrature of the max density
def _max_normal_moments(n: int):
    xs = np.linspace(-8, 8, 16001)
    pdf = np.exp(-xs * xs / 2) / math.sqrt(2 * math.pi)
    cdf = 0.5 * (1 + np.vectorize(math.erf)(xs / math.sqrt(2)))
    dens = n * pdf * cdf ** (n - 1)
    dx = xs[1] - xs[0]
    m = (xs * dens).sum() * dx
    v = (xs * xs * dens).sum() * dx - m * m
    return m, v


_MAXM = {n: _max_normal_moments(n) for n in (25, 81, 169)}

# target: on U[0,1) images roughly DETECT_RATE of anchors have best-class score > 0.25
DETECT_Z = 5.5
SPPF_SHIFT = (2.7, 3.7, 4.2)
SPPF_VAR = (1.45, 1.27, 1.12)
ATTN_VAR = 0.6
VAR_INFLATE = 1.0
VAR_INFLATE_1x1 = 1.2


def calibrate(graph, sd: Dict[str, np.ndarray], in_mean: float = 0.5, in_var: float = 1.0 / 12.0) -> None:
    stats: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
    inb = graph.input
    stats[inb.id] = (np.full(inb.C, in_mean), np.full(inb.C, in_var))

    def get(v):
        m, s = stats[v.buf.id]
        return m[v.coff:v.coff + v.C], s[v.coff:v.coff + v.C]

    def put(v, m, s):
        b = v.buf
        if b.id not in stats:
            stats[b.id] = (np.zeros(b.C), np.ones(b.C))
        stats[b.id][0][v.coff:v.coff + v.C] = m
        stats[b.id][1][v.coff:v.coff + v.C] = s

    for op in graph.ops:
        a = op.args
        if op.kind == "conv":
            m0, v0 = get(a["src0"])
            if a["src1"] is not None:
                m1, v1 = get(a["src1"])
                m0, v0 = np.concatenate([m0, m1]), np.concatenate([v0, v1])
            key = a["wkey"]
            if a.get("convT"):
                w = sd[key + ".weight"].astype(np.float64)  # (in, out, 2, 2)
                b = sd[key + ".bias"].astype(np.float64)
                mo = np.einsum("iokl,i->o", w, m0) / 4 + b
                vo = np.einsum("iokl,i->o", w * w, v0) / 4
                put(a["dst"], mo[: a["dst"].C], vo[: a["dst"].C])
                continue
            w = sd[key + (".conv.weight" if a["bn"] else ".weight")].astype(np.float64)
            wsum = w.sum((2, 3))
            wsq = (w * w).sum((2, 3))
            mo = wsum @ m0
            vo = wsq @ v0 * (VAR_INFLATE if a["k"] == 3 else VAR_INFLATE_1x1)
            if a["bn"]:
                sd[key + ".bn.running_mean"] = mo.astype(np.float32)
                sd[key + ".bn.running_var"] = np.maximum(vo, 1e-3).astype(np.float32)
                g = sd[key + ".bn.weight"].astype(np.float64)
                be = sd[key + ".bn.bias"].astype(np.float64)
                mo, vo = be, g * g * vo / (vo + 1e-3)
            else:
                kind = "cls" if key.split(".")[-2] in () else None
                bias_name = key + ".bias"
                if ".cv3." in key:  # class logits: place the bias DETECT_Z std below the conf=0.25 logit
                    thr = math.log(0.25 / 0.75)
                    sd[bias_name] = (thr - DETECT_Z * np.sqrt(vo) - mo).astype(np.float32)
                mo = mo + sd[bias_name].astype(np.float64)
            if a["act"]:
                mo, vo = _silu_moments(mo, vo)
            if a["res"] is not None:
                rm, rv = get(a["res"])
                mo, vo = mo + rm, vo + rv
            if a["anchor_level"] < 0:
                put(a["dst"], mo, vo)
        elif op.kind == "dwconv":
            m0, v0 = get(a["src"])
            key = a["wkey"]
            w = sd[key + ".conv.weight"].astype(np.float64)[:, 0]
            mo, vo = w.sum((1, 2)) * m0, (w * w).sum((1, 2)) * v0
            sd[key + ".bn.running_mean"] = mo.astype(np.float32)
            sd[key + ".bn.running_var"] = np.maximum(vo, 1e-3).astype(np.float32)
            g = sd[key + ".bn.weight"].astype(np.float64)
            mo, vo = sd[key + ".bn.bias"].astype(np.float64), g * g * vo / (vo + 1e-3)
            if a["act"]:
                mo, vo = _silu_moments(mo, vo)
            put(a["dst"], mo, vo)
        elif op.kind == "sppf":
            m0, v0 = get(a["src"])
            C = a["C"]
            s0 = np.sqrt(v0)
            for j in range(3):
                # SiLU outputs are right-skewed: window maxima shift by ~2.7/3.7/4.2 sigma (measured once on the
                # synthetic graph; see DESIGN.md "synthetic weights")
                put(type(a["src"])(a["dst"], (j + 1) * C, C), m0 + SPPF_SHIFT[j] * s0, v0 * SPPF_VAR[j])
        elif op.kind == "attn":
            mq, vq = get(a["qkv"])
            nh, kd, hd = a["nh"], a["kd"], a["hd"]
            per = 2 * kd + hd
            vm = np.concatenate([mq[h * per + 2 * kd:(h + 1) * per] for h in range(nh)])
            vv = np.concatenate([vq[h * per + 2 * kd:(h + 1) * per] for h in range(nh)])
            key = a["wkey"]
            w = sd[key + ".conv.weight"].astype(np.float64)[:, 0]
            pm, pv = w.sum((1, 2)) * vm, (w * w).sum((1, 2)) * vv
            sd[key + ".bn.running_mean"] = pm.astype(np.float32)
            sd[key + ".bn.running_var"] = np.maximum(pv, 1e-3).astype(np.float32)
            g = sd[key + ".bn.weight"].astype(np.float64)
            pm, pv = sd[key + ".bn.bias"].astype(np.float64), g * g * pv / (pv + 1e-3)
            # softmax-weighted average of v over N keys keeps the mean and shrinks the variance
            put(a["dst"], vm + pm, ATTN_VAR * vv + pv)


def synth_weights(scale: str = "n", task: str = "detect", seed: int = 0) -> Dict[str, np.ndarray]:
    """Ultralytics-style state dict of synthetic weights with calibrated BN stats for yolo11{scale}[-seg]."""
    from .arch import GraphBuilder
    g = GraphBuilder(scale, task)
    sd = synth_state_dict([(p.name, p.shape, p.kind, p.extra) for p in g.params], seed)
    calibrate(g, sd)
    return sd
