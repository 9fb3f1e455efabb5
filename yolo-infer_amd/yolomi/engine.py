"""Engine: one packed YOLO11 model on one GPU, driven through the C-ABI (one graph replay per batch).

PyTorch is plumbing here: it owns the input/output device tensors and the current HIP stream; every arithmetic op
of the forward runs in libyolomi's gfx950 kernels.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from .arch import GraphBuilder
from .lib import Runtime
from .plan import pack_graph


class Engine:
    def __init__(self, scale: str, task: str, state_dict: Dict[str, np.ndarray], device: torch.device,
                 dtype: str = "f16", blob: Optional[bytes] = None):
        if device.type != "cuda":
            raise RuntimeError(f"the yolomi engine runs on a gfx950 GPU (got device {device}); there is no CPU path")
        self.scale, self.task, self.dtype = scale, task, dtype
        self.device = device
        self.graph = GraphBuilder(scale, task)
        self.blob = blob if blob is not None else pack_graph(self.graph, state_dict, dtype)
        self.rt = Runtime(device.index if device.index is not None else torch.cuda.current_device(), self.blob)
        self.nm = self.graph.nm
        self._out: Dict[int, tuple] = {}
        # per-shape on-device autotuning of the conv tiles (ym_tune) on the first call of each (B, H, W)
        self.autotune = os.environ.get("YM_AUTOTUNE", "1") != "0"
        self._tuned = set()

    def outputs(self, B: int, max_det: int):
        key = (B, max_det)
        if key not in self._out:
            dets = torch.zeros((B, max_det, 6 + self.nm), dtype=torch.float32, device=self.device)
            counts = torch.zeros((B,), dtype=torch.int32, device=self.device)
            self._out[key] = (dets, counts)
        return self._out[key]

    def run(self, x: torch.Tensor, conf=0.25, iou=0.7, max_det=300, classes: Optional[Sequence[int]] = None,
            agnostic=False, in_eps=None, use_graph=True, max_nms=30000, max_wh=7680.0):
        """x: (B,3,H,W) float32 contiguous on this device. Returns the engine-owned (dets, counts) tensors."""
        assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4 and x.shape[1] == 3
        B, _, H, W = x.shape
        if in_eps is None:
            in_eps = torch.finfo(torch.float32).eps
        args = Runtime.make_args(conf, iou, max_det, max_nms, agnostic, max_wh, in_eps, classes, use_graph)
        dets, counts = self.outputs(B, max_det)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if self.autotune and (B, H, W) not in self._tuned:
            self.rt.tune(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)
            self._tuned.add((B, H, W))
        self.rt.infer(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)
        return dets, counts

    def profile(self, x: torch.Tensor, **kw):
        B, _, H, W = x.shape
        args = Runtime.make_args(use_graph=False, **kw)
        dets, counts = self.outputs(B, args.max_det)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        return self.rt.profile(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), stream)

    def read_buffer(self, buf_id: int, B: int) -> torch.Tensor:
        """NHWC contents of plan buffer `buf_id` for the first B images (after run/profile), as a CPU float32 tensor."""
        _, C, H, W, eb = self.rt.buffer_info(buf_id)
        dt = torch.float16 if eb == 2 else torch.float32
        out = torch.empty((B, H, W, C), dtype=dt)
        torch.cuda.synchronize(self.device)
        self.rt.read_buffer(buf_id, out.data_ptr(), out.numel() * out.element_size())
        return out.float()
