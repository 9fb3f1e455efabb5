"""Post-training int8 quantisation for the MI355X path: calibration on the GPU and the int8 blob's parameters.

Replaces the reference's `PostTrainingQuantizer` internals (/root/reference/optimization/quantization/quantizers.py):
  * qconfig (:124-131, default backend 'qnnpack' :42): activations HistogramObserver (quint8, per-tensor affine;
    reduce_range on fbgemm), weights MinMaxObserver (qint8, per-tensor symmetric; per-channel on fbgemm) — the same
    torch.ao observer classes, run on the host over tensors produced on the GPU;
  * `_calibrate_model` (:146-177): forward passes over the calibration batches — here the exact-f32 plan of this
    library (`ym_calibrate` also hands back every conv's pre-activation output for the conv-output observers);
  * `convert` (:77): `yolomi.plan.pack_graph(..., dtype="i8", qparams)` builds the int8 plan the gfx950 kernels
    run (csrc/ym_conv_i8.hip).
Quantisation points and numerics: DESIGN.md §9 (the oracle's restatement is oracle/quant.py; names are shared).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Tuple

import numpy as np
import torch

# backend -> (activation reduce_range, per-channel w); "fp8" is the e4m3 PTQ plan (dtype "f8", below)
BACKENDS = {"qnnpack": (False, False), "fbgemm": (True, True), "fp8": (False, True)}
F32 = np.float32
E4M3_MAX = 448.0


def qrange(backend: str) -> Tuple[int, int]:
    return 0, (127 if BACKENDS[backend][0] else 255)


def act_observer(backend: str):
    from torch.ao.quantization.observer import HistogramObserver, MinMaxObserver
    if backend == "fp8":  # amax observer: s = max|x| / 448
        return MinMaxObserver(dtype=torch.quint8, qscheme=torch.per_tensor_affine)
    return HistogramObserver(dtype=torch.quint8, qscheme=torch.per_tensor_affine, reduce_range=BACKENDS[backend][0])


# ----------------------------------------------------------------------------------------- fp8 (e4m3) PTQ plan
# The same quantisation points as the int8 plan, with OCP e4m3 codes (gfx950 fp8) in place of affine uint8: a tensor
# has a per-tensor scale s = amax / 448 (zero point 0) and code = e4m3(clamp(v * (1/s), +-448)) (round to nearest
# even), weights per-output-channel e4m3; convs multiply the e4m3 values (widened exactly to fp16) on the f16 MFMA.
# Restated in oracle/quant.py (backend "fp8") with torch.float8_e4m3fn casts; kernels: csrc/ym_quant.h Q8<true>.
def fp8_scale(amax: float) -> float:
    amax = float(amax)
    return float(F32(amax) / F32(E4M3_MAX)) if amax > 0 else float(F32(1.0) / F32(E4M3_MAX))


def e4m3_codes(v: torch.Tensor) -> torch.Tensor:
    """uint8 e4m3 codes of fp32 values already scaled: clamp to +-448, round to nearest even (torch's cast)."""
    return torch.clamp(v.float(), -E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).view(torch.uint8)


def e4m3_table() -> np.ndarray:
    """value of every e4m3 code (0x7f / 0xff are NaN: never produced, read as 0)."""
    t = torch.arange(256, dtype=torch.int32).to(torch.uint8).view(torch.float8_e4m3fn).float().numpy()
    return np.nan_to_num(t, nan=0.0).astype(F32)


def quantize_weight_fp8(w: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Per-output-channel e4m3 weights: s[n] = max|w[n]| / 448, code = e4m3(w * (1/s[n])) -> (uint8 codes, s)."""
    w = np.ascontiguousarray(w, dtype=F32)
    amax = np.abs(w.reshape(w.shape[0], -1)).max(1)
    s = np.array([fp8_scale(a) for a in amax], F32)
    inv = (F32(1.0) / s).astype(F32)
    t = torch.from_numpy(w) * torch.from_numpy(inv).view(-1, *([1] * (w.ndim - 1)))
    return e4m3_codes(t).numpy(), s


def post_table_fp8(s: float, act: bool) -> np.ndarray:
    """post[code] = act(e4m3(code) * s) for the 256 codes (SiLU in float64, rounded once, as post_table)."""
    x = (e4m3_table() * F32(s)).astype(F32)
    if act:
        d = x.astype(np.float64)
        x = (d / (1.0 + np.exp(-d))).astype(F32)
    return x.astype(F32)


def quantize_weight(w: np.ndarray, per_channel: bool) -> Tuple[np.ndarray, np.ndarray]:
    """torch.ao weight observer + quantize over axis 0 (output channels): (int8 array, fp32 scale per channel)."""
    from torch.ao.quantization.observer import MinMaxObserver, PerChannelMinMaxObserver
    t = torch.from_numpy(np.ascontiguousarray(w, dtype=np.float32))
    if per_channel:
        obs = PerChannelMinMaxObserver(ch_axis=0, dtype=torch.qint8, qscheme=torch.per_channel_symmetric)
        obs(t)
        s, z = obs.calculate_qparams()
        q = torch.quantize_per_channel(t, s.double(), z.long(), 0, torch.qint8).int_repr().numpy()
        return q.astype(np.int8), s.float().numpy().astype(F32)
    obs = MinMaxObserver(dtype=torch.qint8, qscheme=torch.per_tensor_symmetric)
    obs(t)
    s, _ = obs.calculate_qparams()
    q = torch.quantize_per_tensor(t, float(s), 0, torch.qint8).int_repr().numpy()
    return q.astype(np.int8), np.full(w.shape[0], F32(float(s)), F32)


def post_table(s: float, z: int, act: bool) -> np.ndarray:
    """post[q] = act((q - z)·s) for q in [0, 256): the dequantised (and SiLU'd, in float64 rounded once) conv output."""
    x = (np.arange(256, dtype=np.int64) - int(z)).astype(F32) * F32(s)
    if act:
        d = x.astype(np.float64)
        x = (d / (1.0 + np.exp(-d))).astype(F32)
    return x.astype(F32)


def inv32(s: float) -> float:
    return float(F32(1.0) / F32(s))


# --------------------------------------------------------------------------------------------- GPU calibration
class _Observers:
    def __init__(self, backend: str):
        self.backend = backend
        self.obs: Dict[str, object] = {}

    def __call__(self, key: str, t: torch.Tensor):
        o = self.obs.get(key)
        if o is None:
            o = self.obs[key] = act_observer(self.backend)
        o(t.detach().float().cpu())

    def qparams(self) -> Dict:
        qp = {"backend": self.backend}
        for k, o in self.obs.items():
            if self.backend == "fp8":
                qp[k] = (fp8_scale(max(abs(float(o.min_val)), abs(float(o.max_val)))), 0)
                continue
            s, z = o.calculate_qparams()
            qp[k] = (float(F32(float(s))), int(z))
        return qp


def _view(t: torch.Tensor, coff: int, C: int) -> torch.Tensor:
    return t[..., coff:coff + C]


@torch.no_grad()
def calibrate(engine, batches: Iterable[torch.Tensor], backend: str = "qnnpack") -> Dict:
    """Observe every quantisation point of the int8 plan over the calibration batches, running the exact-f32 plan
    (`engine`: a yolomi Engine with dtype 'f32').  Returns {"backend", "act:<tensor>"|"out:<conv>": (scale, zp)}."""
    if engine.dtype != "f32":
        raise ValueError("calibration runs on the exact-f32 plan (Engine dtype 'f32')")
    g = engine.graph
    ob = _Observers(backend)
    for x in batches:
        x = x.to(engine.device).float().contiguous()
        if x.dim() == 3:
            x = x.unsqueeze(0)
        B = x.shape[0]
        eps = torch.finfo(torch.float32).eps
        xin = x / 255.0 if float(x.max()) > 1.0 + eps else x  # LoadTensor (the image as the stem sees it)
        ob("act:input", xin)
        raws = engine.calibrate(x)
        for i, op in enumerate(g.ops):
            if i in raws:
                ob("out:" + op.args["wkey"], raws[i])
        bufs = {}
        for b in g.buffers:
            if b.qname and b.qkind == "act" and b is not g.input:
                bufs[b.id] = engine.read_buffer(b.id, B)  # (B, H, W, C) fp32 on the host
                ob(b.qkey, bufs[b.id])
        for op in g.ops:  # concats that the float plan never materialises (two-source A loaders)
            a = op.args
            if op.kind == "conv" and a.get("catq"):
                s0 = bufs.get(a["src0"].buf.id)
                if s0 is None:
                    s0 = bufs[a["src0"].buf.id] = engine.read_buffer(a["src0"].buf.id, B)
                s1 = bufs.get(a["src1"].buf.id)
                if s1 is None:
                    s1 = bufs[a["src1"].buf.id] = engine.read_buffer(a["src1"].buf.id, B)
                p0 = _view(s0, a["src0"].coff, a["src0"].C)
                if a["up0"]:
                    p0 = p0.repeat_interleave(2, 1).repeat_interleave(2, 2)
                ob("act:" + a["catq"], torch.cat([p0, _view(s1, a["src1"].coff, a["src1"].C)], -1))
    return ob.qparams()
