"""Engine: one packed YOLO11 model on one GPU, driven through the C-ABI (one graph replay per batch).

PyTorch is plumbing here: it owns the input/output device tensors and the current HIP stream; every arithmetic op
of the forward runs in libyolomi's gfx950 kernels.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from .arch import GraphBuilder
from .lib import Runtime
from .plan import QUANT_DTYPES, fuse_default, pack_graph

# Bump when the meaning of a conv config index (csrc/ym_conv.hip kCfgs) changes: stale tables are then ignored.
TUNE_VERSION = 11  # 11: split-pair cfgs encoded kSplitTag + 256·a + b (8 bits per config)
TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")  # committed tables


def tune_cache_dir() -> str:
    return os.environ.get("YM_TUNE_DIR", os.path.join(os.path.expanduser("~"), ".cache", "yolomi", "tune"))


class Engine:
    def __init__(self, scale: str, task: str, state_dict: Dict[str, np.ndarray], device: torch.device,
                 dtype: str = "f16", blob: Optional[bytes] = None, qparams: Optional[Dict] = None, nc: int = 80,
                 receive: Optional[tuple] = None):
        """dtype: 'x3' (split-f16 MFMA, the f16-tolerance plan), 'f16' (throughput), 'f32' (exact parity mode),
        'i8' (PTQ int8) or 'f8' (PTQ fp8 e4m3); the quantized plans need `qparams` from yolomi.quant.calibrate
        (backend 'fp8' for 'f8'), or a packed `blob`.  receive = (rccl comm, root): this rank's context receives the
        root's blob over RCCL (ym_broadcast_weights, a collective the root joins with broadcast_weights())."""
        if device.type != "cuda":
            raise RuntimeError(f"the yolomi engine runs on a gfx950 GPU (got device {device}); there is no CPU path")
        self.scale, self.task, self.dtype = scale, task, dtype
        self.device = device
        self.qparams = qparams
        self.graph = GraphBuilder(scale, task, nc=nc, quant=dtype in QUANT_DTYPES,
                                  fuse=fuse_default(dtype))
        dev_index = device.index if device.index is not None else torch.cuda.current_device()
        if isinstance(receive, Runtime):  # a context that already received the root's blob (yolomi.dist)
            if receive.n_ops != len(self.graph.ops) or receive.device_index != dev_index:
                raise ValueError("the received context does not hold this plan on this device")
            self.blob = None
            self.rt = receive
        elif receive is not None:  # a non-root rank: the model arrives over RCCL from the root's context
            self.blob = None
            self.rt = Runtime(dev_index, None, scale=scale, task=task, dtype=dtype)
            self.rt.broadcast_weights(receive[0], receive[1], torch.cuda.current_stream(device).cuda_stream)
        else:
            self.blob = blob if blob is not None else pack_graph(self.graph, state_dict, dtype, qparams)
            self.rt = Runtime(dev_index, self.blob, scale=scale, task=task, dtype=dtype)
        self.nm = self.graph.nm
        self._out: Dict[int, tuple] = {}
        # Per-shape conv tile tables: on the first call of each (B, H, W) a table is taken from the writable tune
        # cache or the committed `tuned/` directory; failing both, ym_tune measures one on this GPU (and caches it).
        # The exact-f32 parity plan is never autotuned: its tiles (and so its fp32 summation orders) stay the fixed
        # heuristic ones, so its results are reproducible from run to run.
        self.autotune = os.environ.get("YM_AUTOTUNE", "1") != "0" and dtype != "f32"
        # Lanes: the batch runs as up to 4 concurrent image slices (parallel branches of one graph); conv tables are
        # per slice batch.  Default from YM_LANES (1).
        self.lanes = int(os.environ.get("YM_LANES", "1"))
        self._tuned = set()
        self._args_cache = {}
        self.tune_source: Dict[tuple, str] = {}

    def broadcast_weights(self, comm: int, root: int = 0):
        """The root's side of the RCCL weight broadcast (ym_broadcast_weights): every rank of `comm` calls it or
        constructs its Engine with receive=(comm, root)."""
        self.rt.broadcast_weights(comm, root, torch.cuda.current_stream(self.device).cuda_stream)

    def _table_name(self, B, H, W):
        return f"{self.scale}-{self.task}-{self.dtype}-b{B}-{H}x{W}.json"

    def _load_table(self, B, H, W):
        """The committed table first (the one the tests and the bench pin), then this machine's tune cache — so a
        table this machine tuned (ym_tune) for a shape that also has a committed table is cached but not read back
        unless YM_PREFER_CACHE=1 puts the cache first.  A table is used only when its version, op-name list, device
        architecture and conv-config catalogue size (ym_num_conv_cfgs: the id space its entries index) all match."""
        name = self._table_name(B, H, W)
        arch = torch.cuda.get_device_properties(self.device).gcnArchName
        ops = [op.name for op in self.graph.ops]
        order = [("committed", TUNED_DIR), ("cache", tune_cache_dir())]
        if os.environ.get("YM_PREFER_CACHE", "0") == "1":
            order.reverse()
        for tag, d in order:
            p = os.path.join(d, name)
            try:
                t = json.load(open(p))
            except (OSError, ValueError):
                continue
            dev = t.get("device")
            if (t.get("version") == TUNE_VERSION and t.get("ops") == ops and len(t.get("cfg", [])) == self.rt.n_ops
                    and t.get("ncfg") == self._ncfg() and (dev is None or dev.split(":")[0] == arch.split(":")[0])):
                self.rt.set_op_cfg(B, H, W, t["cfg"])
                return f"{tag} table {name}"
        return None

    def _ncfg(self) -> int:
        from yolomi.lib import DTYPE_CODES, load_library
        return load_library().ym_num_conv_cfgs(DTYPE_CODES[self.dtype])

    def _save_table(self, B, H, W):
        cfg = self.rt.get_op_cfg(B, H, W)
        if cfg is None:
            return
        d = tune_cache_dir()
        try:
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, self._table_name(B, H, W)), "w") as f:
                json.dump({"version": TUNE_VERSION, "device": torch.cuda.get_device_properties(self.device).gcnArchName,
                           "ncfg": self._ncfg(), "ops": [op.name for op in self.graph.ops], "cfg": cfg}, f)
        except OSError:
            pass  # a read-only home: the table lives for this process only

    def _prepare_shape(self, x, B, H, W, args, dets, counts, stream):
        src = None if os.environ.get("YM_TUNE_TABLES", "1") == "0" else self._load_table(B, H, W)
        if src is None and self.autotune:
            self.rt.tune(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)
            self._save_table(B, H, W)
            src = "ym_tune"
        self.tune_source[(B, H, W)] = src or "heuristic"
        self._tuned.add((B, H, W))

    def outputs(self, B: int, max_det: int):
        key = (B, max_det)
        if key not in self._out:
            dets = torch.zeros((B, max_det, 6 + self.nm), dtype=torch.float32, device=self.device)
            counts = torch.zeros((B,), dtype=torch.int32, device=self.device)
            self._out[key] = (dets, counts)
        return self._out[key]

    def rows_buffer(self, B: int, max_det: int):
        """A fresh flat fp32 device buffer for one call: (rows (B, max_det, 6 + nm) view, counts (B,) int32 view of the
        words behind the rows) — for run(..., dets_out=rows, counts_after=True)."""
        no = 6 + self.nm
        flat = torch.empty((B * max_det * no + B,), dtype=torch.float32, device=self.device)
        return flat[: B * max_det * no].view(B, max_det, no), flat[B * max_det * no:].view(torch.int32)

    def lane_batch(self, B: int, lanes: Optional[int] = None) -> int:
        """Images per lane (the batch every kernel sees) for a B-image call: ceil(B / clamp(lanes, 1, 4, B))."""
        L = max(1, min(self.lanes if lanes is None else lanes, 4, B))
        return -(-B // L)

    def run(self, x: torch.Tensor, conf=0.25, iou=0.7, max_det=300, classes: Optional[Sequence[int]] = None,
            agnostic=False, in_eps=None, use_graph=True, max_nms=30000, max_wh=7680.0, lanes=None,
            batch_max: Optional[torch.Tensor] = None, dets_out: Optional[torch.Tensor] = None,
            counts_after: bool = False):
        """x: (B,3,H,W) float32 contiguous on this device. Returns the engine-owned (dets, counts) tensors, or
        (dets_out, counts) when the caller hands in its own (>= B, max_det, 6 + nm) fp32 rows (predict(): a fresh
        tensor per call, written by the NMS kernel directly — a cached graph re-points its NMS nodes, no copy).
        batch_max: optional (1,) fp32 device tensor, the max over the GLOBAL batch (yolomi.dist: a batch-sharded
        rank takes LoadTensor's /255 decision from it instead of from its own shard).
        counts_after (with dets_out = the first B*max_det rows of a flat buffer, see rows_buffer): the NMS also writes
        this call's B detection counts as int32 words right behind those rows, so the caller can read them later
        (predict() reads them lazily: no host sync per call)."""
        assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4 and x.shape[1] == 3
        B, _, H, W = x.shape
        if in_eps is None:
            in_eps = torch.finfo(torch.float32).eps
        lanes = self.lanes if lanes is None else lanes
        # the ctypes argument block of a repeated call is reused (predict loops pass the same thresholds)
        bm = 0
        if batch_max is not None:
            assert batch_max.is_cuda and batch_max.dtype == torch.float32 and batch_max.numel() >= 1
            bm = batch_max.data_ptr()
        akey = (conf, iou, max_det, max_nms, agnostic, max_wh, in_eps, tuple(classes) if classes is not None else None,
                use_graph, lanes, bm, counts_after)
        args = self._args_cache.get(akey)
        if args is None:
            if len(self._args_cache) > 64:
                self._args_cache.clear()
            args = self._args_cache[akey] = Runtime.make_args(conf, iou, max_det, max_nms, agnostic, max_wh, in_eps,
                                                              classes, use_graph, lanes, bm, counts_after)
        dets, counts = self.outputs(B, max_det)
        if dets_out is not None:
            assert (dets_out.is_cuda and dets_out.dtype == torch.float32 and dets_out.is_contiguous()
                    and dets_out.dim() == 3 and dets_out.shape[0] >= B and tuple(dets_out.shape[1:]) == tuple(dets.shape[1:]))
            dets = dets_out
        if counts_after:  # room for the B count words behind the rows, in dets_out's own storage
            need = dets_out.storage_offset() * 4 + B * max_det * (6 + self.nm) * 4 + 4 * B if dets_out is not None else -1
            if dets_out is None or dets_out.untyped_storage().nbytes() < need:
                raise ValueError("counts_after needs dets_out from Engine.rows_buffer (rows followed by B int32 words)")
        stream = torch.cuda.current_stream(self.device).cuda_stream
        Bl = self.lane_batch(B, lanes)
        if (Bl, H, W) not in self._tuned:
            self._prepare_shape(x[:Bl], Bl, H, W, args, dets, counts, stream)
        self.rt.infer(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)
        return dets, counts

    def input_max(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(1,) fp32 device tensor: max over x (LoadTensor's statistic; asynchronous on the current stream)."""
        assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
        if out is None:
            out = torch.empty((1,), dtype=torch.float32, device=self.device)
        self.rt.input_max(x.data_ptr(), x.numel(), out.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        return out

    def profile(self, x: torch.Tensor, **kw):
        B, _, H, W = x.shape
        args = Runtime.make_args(use_graph=False, **kw)
        dets, counts = self.outputs(B, args.max_det)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if (B, H, W) not in self._tuned:
            self._prepare_shape(x, B, H, W, args, dets, counts, stream)
        return self.rt.profile(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)

    def profile_replay(self, x: torch.Tensor, reps=20, **kw):
        """Per-op device ms from graph-captured back-to-back launches (-1 for input/decode/NMS); clobbers buffers."""
        B, _, H, W = x.shape
        args = Runtime.make_args(use_graph=False, **kw)
        dets, counts = self.outputs(B, args.max_det)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if (B, H, W) not in self._tuned:
            self._prepare_shape(x, B, H, W, args, dets, counts, stream)
        return self.rt.profile_replay(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream, reps)

    def masks(self, dets: torch.Tensor, counts: Sequence[int], H: int, W: int):
        """Segment plans: instance masks of the last run()'s detections (process_mask, upsample=True).  Returns the
        (total, H, W) uint8 masks, the (total,) int32 non-empty flags and the per-image row offsets (host list)."""
        B = len(counts)
        offs = [0]
        for n in counts:
            offs.append(offs[-1] + int(n))
        total = offs[-1]
        masks = torch.empty((total, H, W), dtype=torch.uint8, device=self.device)
        nonempty = torch.empty((total,), dtype=torch.int32, device=self.device)  # zeroed by ym_masks
        if total:
            off_t = torch.tensor(offs, dtype=torch.int32).to(self.device, non_blocking=True)
            stream = torch.cuda.current_stream(self.device).cuda_stream
            self.rt.masks(dets.data_ptr(), B, dets.shape[1], off_t.data_ptr(), total, H, W, masks.data_ptr(),
                          nonempty.data_ptr(), stream)
        return masks, nonempty, offs

    def masks_slots(self, dets: torch.Tensor, counts: torch.Tensor, cap: int, H: int, W: int):
        """Single-sync form of masks(): enqueued behind the forward, reading the DEVICE counts.  Returns the
        (B, cap, H, W) uint8 masks (slot (b, i) = detection i of image b, for i < min(count_b, cap)) and a (B*cap + B)
        int32 tensor: the slots' non-empty flags, then the B counts (read both with one .tolist())."""
        B = counts.shape[0]
        masks = torch.empty((B, cap, H, W), dtype=torch.uint8, device=self.device)
        flags = torch.empty((B * cap + B,), dtype=torch.int32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.rt.masks_slots(dets.data_ptr(), B, dets.shape[1], counts.data_ptr(), cap, H, W, masks.data_ptr(),
                            flags.data_ptr(), stream)
        return masks, flags

    def read_buffer(self, buf_id: int, B: int, raw: bool = False) -> torch.Tensor:
        """NHWC contents of plan buffer `buf_id` for the first B images (after run/profile), as a CPU float32 tensor
        (int8 plans: the quantized values q = stored byte + 128; fp8 plans: the e4m3 values of the stored codes;
        over the storage channels).  raw=True: the stored elements as they are (int8 / fp16 / fp32 tensor)."""
        _, C, H, W, eb = self.rt.buffer_info(buf_id)
        dt = {1: torch.int8, 2: torch.float16, 4: torch.float32}[eb]
        pair = self.dtype == "x3" and not self.graph.buffers[buf_id].f32
        if pair:  # x3 pair layout: every 8-channel chunk is [fp16 hi x8 | fp16 lo x8]
            dt = torch.float16
        out = torch.empty((B, H, W, 2 * C if pair else C), dtype=dt)
        torch.cuda.synchronize(self.device)
        self.rt.read_buffer(buf_id, out.data_ptr(), out.numel() * out.element_size())
        if pair:
            if raw:
                return out
            hl = out.float().reshape(B, H, W, C // 8, 2, 8)
            return (hl[..., 0, :] + hl[..., 1, :]).reshape(B, H, W, C)
        if raw or eb != 1:
            return out if raw else out.float()
        if self.dtype == "f8":
            return out.view(torch.uint8).view(torch.float8_e4m3fn).float()
        return out.float() + 128.0

    def raw_shapes(self, B: int, H: int, W: int) -> Dict[int, tuple]:
        """(rows, cols) of every op's pre-activation output in a calibration run (ym_calibrate)."""
        shapes = {}
        for i, op in enumerate(self.graph.ops):
            a = op.args
            if op.kind == "conv":
                fo = self.graph.out_factor(op)
                shapes[i] = (B * (H // fo) * (W // fo), 4 * a["c2"] if a["shuffle2x2"] else a["c2"])
            elif op.kind == "dwconv":
                f = a["src"].buf.f
                shapes[i] = (B * (H // f) * (W // f), a["C"])
            elif op.kind == "attn":
                f = a["qkv"].buf.f
                shapes[i] = (B * (H // f) * (W // f), a["C"])
        return shapes

    def calibrate(self, x: torch.Tensor, **kw) -> Dict[int, torch.Tensor]:
        """One eager f32 forward that also returns every conv-like op's pre-activation output (op index → (rows, C)
        fp32 device tensor): the conv-output observers of PTQ calibration (yolomi.quant.calibrate)."""
        assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4
        B, _, H, W = x.shape
        args = Runtime.make_args(use_graph=False, lanes=1, **kw)
        dets, counts = self.outputs(B, args.max_det)
        raws = {i: torch.empty(sh, dtype=torch.float32, device=self.device)
                for i, sh in self.raw_shapes(B, H, W).items()}
        ptrs = [raws[i].data_ptr() if i in raws else 0 for i in range(len(self.graph.ops))]
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.rt.calibrate(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), ptrs, stream)
        torch.cuda.synchronize(self.device)
        return raws
