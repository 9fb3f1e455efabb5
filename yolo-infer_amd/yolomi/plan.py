"""Model blob packer: Ultralytics-style state dict + YOLO11 plan → one binary blob for `ym_load_weights`.

Replaces what Ultralytics' AutoBackend(fuse=True) does on first predict: Conv+BN folding
(`fuse_conv_and_bn`, restated bit-for-bit in fp32: W' = (γ/√(eps+σ²))·W, b' = β − γ·μ/√(σ²+eps)), then — the MI355X
part — packing every conv as a K-contiguous GEMM B operand [N][Kpad] with K ordered (ky, kx, c) to match the NHWC
implicit-GEMM loader (`csrc/ym_conv.hip`), the stem's Cin padded 3→8, ConvTranspose2d(2,2) re-laid out as a 1x1
GEMM with N = 4·C (pixel-shuffle epilogue), depthwise weights as [9][C] fp32.

int8 plans (dtype "i8", the runtime of the reference's PostTrainingQuantizer.convert,
`optimization/quantization/quantizers.py:77`): weights quantized with the torch.ao observer of the calibrated
backend, K padded to 16-channel granules per tap, and per op a `QRec` (csrc/ym_common.h: requantisation of the conv
output, the 256-entry post-activation table, the stored tensor's / residual's / input's quantisation), the fp32
s_in·s_w per output channel and the int32 zero-point correction Σ_k (128 - z_in)·w (activations are stored as q - 128).

x3 plans (dtype "x3", the parity plan benched): activations in the pair layout of csrc/ym_common.h (every 8-channel
chunk as fp16 hi = fp16(x) then lo = fp16(x - hi)); every conv weight row except the stem's likewise, [hi x8 | lo x8]
per K chunk, of the weights scaled by a power of two 2^s (max |w·2^s| in (2^13, 2^14], so the lo parts stay normal;
s in record slot 22, W2's in slot 23), so r[21] (Kpad) counts fp16 storage elements: 2·K padded to 64.  The stem
keeps fp32 rows.

Blob layout (int32 little-endian; parsed by `csrc/ym_runtime.cpp:ym_load_weights`):
  header[32] | buffers[nbuf][8] | ops[nop][32] | names[nop][48 bytes] | pad to 256 | weights
Conv op record: [1..5] k, s, Cin, N, act | [6..9] src0 buf, coff, C, up0 | [10..12] src1 | [13..16] dst buf, coff,
anchor level, pixel shuffle | [17..18] residual | [19..21] weight / bias offsets, Kpad | [22..24] int8 QRec, s_in·s_w,
int32 bias (f16 / x3 plans: r[24] = 1 + offset of a fused depthwise's [9][C] weights ‖ [C] bias, GraphBuilder.fuse_dw;
0: none) | [25..31] fused successor conv (f16 plans, GraphBuilder.fuse_pairs): W2 / bias2 offsets, N2, act2, Kpad2,
its kernel size k2 (1: streaming FUSE; 3: Bottleneck kernel), intermediate buffer (used when the tuner runs the pair as
two launches).
"""
from __future__ import annotations

import struct
from typing import Dict, List

import numpy as np

from .arch import REG_MAX, STRIDES, GraphBuilder

MAGIC = 0x4C504D59
VERSION = 1
OP_IDS = {"input": 1, "conv": 2, "dwconv": 3, "sppf": 4, "attn": 5, "decode": 6, "nms": 7, "requant": 8}
DTYPES = {"f16": 0, "f32": 1, "i8": 2, "f8": 3, "x3": 4}
QUANT_DTYPES = ("i8", "f8")  # one-byte PTQ plans: int8 affine (torch.ao qconfig) and fp8 e4m3 (yolomi/quant.py)
BK = 64  # conv K is padded to the kernel K step (csrc/ym_conv.hip KSTEP)


def fuse_conv_bn(w: np.ndarray, gamma, beta, mean, var, eps=1e-3):
    """ultralytics.utils.torch_utils.fuse_conv_and_bn in fp32 (bit-identical to the torch CPU path)."""
    f = np.float32
    w = w.astype(f)
    scale = gamma.astype(f) / np.sqrt(f(eps) + var.astype(f))
    wf = (scale.reshape(-1, *([1] * (w.ndim - 1))) * w).astype(f)
    bf = (beta.astype(f) - (gamma.astype(f) * mean.astype(f)) / np.sqrt(var.astype(f) + f(eps))).astype(f)
    return wf, bf


class _WeightArena:
    def __init__(self):
        self.chunks: List[bytes] = []
        self.size = 0

    def add(self, arr: np.ndarray) -> int:
        off = self.size
        b = np.ascontiguousarray(arr).tobytes()
        pad = (-len(b)) % 256
        self.chunks.append(b + b"\0" * pad)
        self.size += len(b) + pad
        return off

    def bytes(self) -> bytes:
        return b"".join(self.chunks)


def _conv_weights(a: dict, sd: Dict[str, np.ndarray]):
    if a.get("wkeys"):  # sibling convs on one input merged into one GEMM (arch.py C3k): output channels concatenated
        parts = [_conv_weights(dict(a, wkeys=None, wkey=k), sd) for k in a["wkeys"]]
        return np.concatenate([w for w, _ in parts]), np.concatenate([b for _, b in parts])
    key = a["wkey"]
    if a.get("convT"):
        wt = sd[key + ".weight"].astype(np.float32)  # (in, out, 2, 2)
        cin, cout = wt.shape[0], wt.shape[1]
        # GEMM column n = (dy*2 + dx)*cout + o  ←  wt[c, o, dy, dx]
        wg = np.transpose(wt, (2, 3, 1, 0)).reshape(4 * cout, cin)
        bg = np.tile(sd[key + ".bias"].astype(np.float32), 4)
        return wg[:, None, None, :], bg  # (N, 1, 1, cin)
    if a["bn"]:
        w, b = fuse_conv_bn(sd[key + ".conv.weight"], sd[key + ".bn.weight"], sd[key + ".bn.bias"],
                            sd[key + ".bn.running_mean"], sd[key + ".bn.running_var"])
    else:
        w, b = sd[key + ".weight"].astype(np.float32), sd[key + ".bias"].astype(np.float32)
    return np.transpose(w, (0, 2, 3, 1)), b  # (cout, k, k, cin) = NHWC-K order


def _dw_weights(key: str, sd):
    w, b = fuse_conv_bn(sd[key + ".conv.weight"], sd[key + ".bn.weight"], sd[key + ".bn.bias"],
                        sd[key + ".bn.running_mean"], sd[key + ".bn.running_var"])
    C = w.shape[0]
    return np.ascontiguousarray(w.reshape(C, 9).T).astype(np.float32), b  # [9][C]


X3_WEXP_MAX = 64  # |s| the runtime accepts for an x3 weight scale 2^s (csrc/ym_runtime.cpp conv_args)
X3_WMAX_LOG2 = 14  # x3 weight scaling: max |w|·2^s in (2^13, 2^14] (fp16 max 65504; csrc/ym_common.h ConvArgs::wsc)


def x3_weight_exp(w: np.ndarray) -> int:
    """Power-of-two exponent s of an x3 weight matrix: stored as w·2^s so that the fp16 lo part of the split
    (lo = fp16(w·2^s - hi)) stays normal for every weight above 2^-17 of the matrix's max — unscaled, the typical
    folded weight (~0.03) sits where lo is subnormal and keeps ~1e-6 relative precision (tools/x3_emulate.py).
    The kernels multiply the accumulator by 2^-s in the epilogue (exact)."""
    m = float(np.abs(w).max()) if w.size else 0.0
    if not np.isfinite(m):
        raise ValueError("non-finite conv weight")
    if m == 0.0:
        return 0
    # clamped to the range ym_load_weights accepts (conv_args: |s| <= X3_WEXP_MAX): a nearly pruned matrix (max |w|
    # below 2^-50) keeps s = 64 and with it subnormal lo parts, instead of a blob the loader rejects
    return int(min(max(X3_WMAX_LOG2 - np.ceil(np.log2(m)), -X3_WEXP_MAX), X3_WEXP_MAX))


def x3_pair_rows(w: np.ndarray, s: int) -> np.ndarray:
    """(N, K) fp32 weights → [N][2K] fp16 pair-chunk rows of w·2^s: every 8-element K chunk as [hi x8 | lo x8]."""
    N, K = w.shape
    wr = (w.astype(np.float32).reshape(N, K // 8, 8) * np.float32(2.0 ** s)).astype(np.float32)
    hi = wr.astype(np.float16)
    lo = (wr - hi.astype(np.float32)).astype(np.float16)
    return np.stack([hi, lo], axis=2).reshape(N, 2 * K)


def _qrec(inv_sc, zc, qlo, qhi, mode, post, inv_so=1.0, zo=0, s_r=0.0, z_r=0, s_in=0.0, z_in=0, inv_s_in=0.0) -> bytes:
    """csrc/ym_common.h `QRec` (1088 bytes)."""
    head = struct.pack("<fiiiifififif4i", inv_sc, int(zc), int(qlo), int(qhi), int(mode), inv_so, int(zo), s_r,
                       int(z_r), s_in, int(z_in), inv_s_in, 0, 0, 0, 0)
    return head + np.asarray(post, np.float32).tobytes()


def fuse_default(dtype: str):
    """GraphBuilder `fuse` of a plan unless YM_FUSE=0: f16 plans fuse conv pairs (GraphBuilder.fuse_pairs) and merge
    C3k's cv1 ‖ cv2; x3 plans merge and fuse the pairs with a 1x1 successor ("x3": GraphBuilder)."""
    import os
    if os.environ.get("YM_FUSE", "1") == "0":
        return False
    return {"f16": True, "x3": "x3"}.get(dtype, False)


def check_state_dict(g: GraphBuilder, sd: Dict[str, np.ndarray]) -> None:
    """Every parameter the plan reads must exist with exactly the shape the graph declares: a checkpoint of another
    scale, task or class count is rejected here instead of being packed with the wrong K pitch / channel count."""
    for p in g.params:
        if p.kind in ("count", "dfl"):
            continue
        if p.name not in sd:
            raise ValueError(f"state dict has no {p.name!r} (plan yolo11{g.scale} {g.task}, nc={g.nc})")
        shape = tuple(np.shape(sd[p.name]))
        if shape != tuple(p.shape):
            raise ValueError(f"{p.name}: checkpoint shape {shape} != plan shape {tuple(p.shape)} "
                             f"(plan yolo11{g.scale} {g.task}, nc={g.nc}: scale/task/class-count mismatch)")


def pack_model(scale: str, task: str, sd: Dict[str, np.ndarray], dtype: str = "f16", qparams: Dict = None) -> bytes:
    g = GraphBuilder(scale, task, quant=dtype in QUANT_DTYPES, fuse=fuse_default(dtype))
    return pack_graph(g, sd, dtype, qparams)


def pack_graph(g: GraphBuilder, sd: Dict[str, np.ndarray], dtype: str = "f16", qparams: Dict = None) -> bytes:
    if dtype not in DTYPES:
        raise ValueError(f"dtype {dtype!r} not in {list(DTYPES)}")
    quant = dtype in QUANT_DTYPES
    f8 = dtype == "f8"
    if quant != bool(g.quant):
        raise ValueError("int8/fp8 blobs need GraphBuilder(quant=True), float blobs quant=False")
    check_state_dict(g, sd)
    if quant:
        from .quant import (BACKENDS, inv32, post_table, post_table_fp8, qrange, quantize_weight,
                            quantize_weight_fp8)
        if not qparams or qparams.get("backend") not in BACKENDS or (qparams["backend"] == "fp8") != f8:
            raise ValueError(f"dtype {dtype!r} needs calibrated qparams (yolomi.quant.calibrate) of backend "
                             f"{'fp8' if f8 else 'qnnpack / fbgemm'}")
        if f8 and g.task != "detect":
            raise ValueError("the fp8 plan covers detect models")
        per_channel = BACKENDS[qparams["backend"]][1]
        qlo, qhi = qrange(qparams["backend"])

        def qweight(w, pc):  # (codes as int8 bytes, fp32 scale per output channel)
            if f8:
                c, sw_ = quantize_weight_fp8(w)
                return c.view(np.int8), sw_
            return quantize_weight(w, pc)

        def post(s_, z_, act):
            return post_table_fp8(s_, act) if f8 else post_table(s_, z_, act)

        def qp(key):
            if key not in qparams:
                raise ValueError(f"qparams has no entry {key!r}")
            s_, z_ = qparams[key]
            return float(np.float32(s_)), int(z_)
    np_dt = np.float16 if dtype == "f16" else np.float32
    arena = _WeightArena()
    op_recs: List[List[int]] = []
    names: List[bytes] = []
    for op in g.ops:
        a = op.args
        r = [0] * 32
        r[0] = OP_IDS[op.kind]
        if op.kind == "conv":
            w, b = _conv_weights(a, sd)  # (N, k, k, cin)
            src0 = a["src0"]
            C0 = src0.C
            stem = src0.buf is g.input
            if quant:
                w, sw = qweight(w, per_channel and not a.get("convT"))  # int8 / e4m3 (N, k, k, cin), fp32 (N,)
            if stem:  # stem: RGB padded to 8 channels
                pad = 8 - C0
                w = np.concatenate([w, np.zeros(w.shape[:3] + (pad,), w.dtype)], axis=3)
                C0 = 8
            elif quant and C0 % 16:  # int8 K chunks are 16 channels of one tap
                pad = 16 - C0 % 16
                w = np.concatenate([w, np.zeros(w.shape[:3] + (pad,), w.dtype)], axis=3)
                C0 += pad
            N = w.shape[0]
            K = w.shape[1] * w.shape[2] * w.shape[3]
            bk = 2 * BK if dtype == "i8" else BK  # int8: whole 128-byte K stages for the LDS-DMA kernels' Q8 mode
            Kpad = (K + bk - 1) // bk * bk
            wp = np.zeros((N, Kpad), np.int8 if quant else np.float32)
            wp[:, :K] = w.reshape(N, K)
            if dtype == "x3" and not stem:  # pair-chunk rows of W·2^s: every 8-channel K chunk as [hi x8 | lo x8]
                ws = x3_weight_exp(w)
                K2 = 2 * K
                Kpad = (K2 + BK - 1) // BK * BK  # the 64-deep storage step (32 logical K)
                wp = np.zeros((N, Kpad), np.float16)
                wp[:, :K2] = x3_pair_rows(w.reshape(N, K), ws)
                r[22] = ws
            src1 = a["src1"]
            C1 = src1.C if src1 is not None else 0
            dst, res = a["dst"], a["res"]
            r[1:6] = [a["k"], a["s"], C0 + C1, N, int(bool(a["act"]))]
            r[6:10] = [src0.buf.id, src0.coff, C0, int(bool(a["up0"]))]
            r[10:13] = [src1.buf.id, src1.coff, C1] if src1 is not None else [-1, 0, 0]
            r[13:17] = [dst.buf.id, dst.coff, a["anchor_level"], int(bool(a["shuffle2x2"]))]
            r[17:19] = [res.buf.id, res.coff] if res is not None else [-1, 0]
            r[19] = arena.add(wp if quant or wp.dtype == np.float16 else wp.astype(np_dt))  # (x3 stem: fp32)
            r[20] = arena.add(b.astype(np.float32))
            r[21] = Kpad
            if a.get("dw") is not None:  # fused depthwise (GraphBuilder.fuse_dw): r[24] = 1 + offset of [9][C] ‖ bias [C]
                if dtype not in ("f16", "x3"):
                    raise ValueError(f"op {op.name}: fused depthwise convs are f16 / x3 only")
                w9, bdw = _dw_weights(a["dw"]["wkey"], sd)
                assert w9.shape == (9, C0)
                r[24] = 1 + arena.add(np.concatenate([w9.reshape(-1), np.asarray(bdw, np.float32)]).astype(np.float32))
            pair = a.get("pair")
            if pair is not None:  # fused successor (GraphBuilder.fuse_pairs): W2 [N2][Kpad2], K = (ky, kx, this conv's N)
                if dtype not in ("f16", "x3"):
                    raise ValueError(f"op {op.name}: fused conv pairs are f16 / x3 only")
                w2, b2 = _conv_weights(pair, sd)  # (N2, k2, k2, N)
                N2, k2 = w2.shape[0], pair["k"]
                assert w2.shape[1:] == (k2, k2, N)
                K2 = k2 * k2 * N
                if dtype == "x3":  # pair-chunk rows of W2·2^s2 like W (storage K 2·K2, padded to 64)
                    ws2 = x3_weight_exp(w2)
                    Kpad2 = (2 * K2 + BK - 1) // BK * BK
                    w2h = np.zeros((N2, Kpad2), np.float16)
                    w2h[:, :2 * K2] = x3_pair_rows(w2.reshape(N2, K2), ws2)
                    r[23] = ws2
                else:
                    Kpad2 = (K2 + BK - 1) // BK * BK
                    w2p = np.zeros((N2, Kpad2), np.float32)
                    w2p[:, :K2] = w2.reshape(N2, K2)
                    w2h = w2p.astype(np.float16)
                r[25], r[26] = arena.add(w2h), arena.add(b2.astype(np.float32))
                r[27:32] = [N2, int(bool(pair["act"])), Kpad2, k2, pair["mid"].buf.id]
            if quant:
                s_in, z_in = qp("act:input" if stem else src0.buf.qkey)
                so, zo = qp("out:" + a["wkey"])
                d = dst.buf
                mode = 2 if d.f32 else (1 if d.qkind == "out" else 0)
                s_b, z_b = (1.0, 0) if mode else qp(d.qkey)
                s_r, z_r = qp(res.buf.qkey) if res is not None else (0.0, 0)
                rec = _qrec(inv32(so), zo, qlo, qhi, mode, post(so, zo, bool(a["act"])), inv32(s_b), z_b, s_r,
                            z_r, s_in, z_in, inv32(s_in))
                biasi = np.zeros(N, np.int64) if (stem or f8) else (128 - z_in) * wp.astype(np.int64).sum(1)
                assert np.abs(biasi).max() < 2 ** 31
                r[22] = arena.add(np.frombuffer(rec, np.uint8))
                r[23] = arena.add((np.float32(s_in) * sw).astype(np.float32))
                r[24] = arena.add(biasi.astype(np.int32))
        elif op.kind == "dwconv":
            w9, b = _dw_weights(a["wkey"], sd)
            r[3], r[5] = a["C"], int(bool(a["act"]))
            r[6], r[7] = a["src"].buf.id, a["src"].coff
            r[13], r[14] = a["dst"].buf.id, a["dst"].coff
            if quant:
                wq, sw = qweight(np.ascontiguousarray(w9.T), per_channel)  # (C, 9): per output channel
                s_in, z_in = qp(a["src"].buf.qkey)
                so, zo = qp("out:" + a["wkey"])
                s_b, z_b = qp(a["dst"].buf.qkey)
                rec = _qrec(inv32(so), zo, qlo, qhi, 0, post(so, zo, bool(a["act"])), inv32(s_b), z_b,
                            s_in=s_in, z_in=z_in)
                r[19], r[20] = arena.add(np.ascontiguousarray(wq.T)), arena.add(b)
                r[22] = arena.add(np.frombuffer(rec, np.uint8))
                r[23] = arena.add((np.float32(s_in) * sw).astype(np.float32))
            else:
                r[19], r[20] = arena.add(w9), arena.add(b)
        elif op.kind == "sppf":
            r[3] = a["C"]
            r[7] = a["src"].coff
            r[13] = a["dst"].id
        elif op.kind == "attn":
            w9, b = _dw_weights(a["wkey"], sd)
            r[3], r[4], r[5], r[9] = a["C"], a["nh"], a["kd"], a["hd"]
            r[6], r[7] = a["qkv"].buf.id, a["qkv"].coff
            r[13], r[14] = a["dst"].buf.id, a["dst"].coff
            r[21] = struct.unpack("<i", struct.pack("<f", float(np.float32(a["kd"] ** -0.5))))[0]
            if quant:
                wq, sw = qweight(np.ascontiguousarray(w9.T), per_channel)
                s_in, z_in = qp(a["qkv"].buf.qkey)
                so, zo = qp("out:" + a["wkey"])
                s_b, z_b = qp(a["dst"].buf.qkey)
                rec = _qrec(inv32(so), zo, qlo, qhi, 0, post(so, zo, False), inv32(s_b), z_b, s_in=s_in,
                            z_in=z_in)
                r[19], r[20] = arena.add(np.ascontiguousarray(wq.T)), arena.add(b)
                r[22] = arena.add(np.frombuffer(rec, np.uint8))
                r[23] = arena.add((np.float32(s_in) * sw).astype(np.float32))
            else:
                r[19], r[20] = arena.add(w9), arena.add(b)
        elif op.kind == "requant":
            src, dst = a["src"], a["dst"]
            r[3] = dst.C
            r[6], r[7], r[9] = src.buf.id, src.coff, int(bool(a["up"]))
            r[13], r[14] = dst.buf.id, dst.coff
            s_in, z_in = qp(src.buf.qkey)
            s_b, z_b = qp(dst.buf.qkey)
            rec = _qrec(1.0, 0, qlo, qhi, 0, np.zeros(256, np.float32), inv32(s_b), z_b, s_in=s_in, z_in=z_in)
            r[22] = arena.add(np.frombuffer(rec, np.uint8))
        op_recs.append(r)
        nm = op.name.encode()[:47]
        names.append(nm + b"\0" * (48 - len(nm)))

    wbytes = arena.bytes()
    hdr = [0] * 32
    hdr[0], hdr[1], hdr[2] = MAGIC, VERSION, DTYPES[dtype]
    hdr[3] = 1 if g.task == "segment" else 0
    hdr[4], hdr[5], hdr[6], hdr[7] = g.nc, g.nm, REG_MAX, len(STRIDES)
    hdr[8:11] = list(STRIDES)
    hdr[11], hdr[12] = len(g.buffers), len(g.ops)
    hdr[13], hdr[14] = len(wbytes) & 0xFFFFFFFF, len(wbytes) >> 32
    hdr[15], hdr[16] = g.input.id, g.anchor_buf.id
    hdr[17] = g.proto_buf.id if g.task == "segment" else -1
    hdr[18] = g.no
    hdr[19] = ord(g.scale)  # checked against ym_model_desc.scale
    head = struct.pack("<32i", *hdr)
    bufs = b"".join(struct.pack("<8i", b.Cs or b.C, b.f, int(b.f32), 0, 0, 0, 0, 0) for b in g.buffers)
    ops = b"".join(struct.pack("<32i", *rr) for rr in op_recs)
    meta = head + bufs + ops + b"".join(names)
    meta += b"\0" * ((-len(meta)) % 256)
    return meta + wbytes
