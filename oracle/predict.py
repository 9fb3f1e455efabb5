"""The oracle's end-to-end predict: restates `YOLO11Model.predict` (`/root/reference/core/model.py:118-133`) for
tensor sources, i.e. Ultralytics BasePredictor.stream_inference → LoadTensor → preprocess (`.float()`) →
DetectionModel forward (fused) → DetectionPredictor.postprocess (NMS → scale_boxes) [→ SegmentationPredictor
process_mask].  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from . import postprocess as pp
from .yolo11 import build


class OracleModel:
    def __init__(self, scale: str, task: str, state_dict: Dict):
        self.scale, self.task = scale, task
        self.net = build(scale, task, state_dict, fuse=True)

    @torch.no_grad()
    def raw(self, im: torch.Tensor, keep=()):
        """Preprocessed forward: returns (y (B, 84[+32], A), extras dict)."""
        im = pp.load_tensor_check(im.float().cpu() if im.dtype != torch.float32 else im.cpu()).float()
        out, saved = self.net(im, keep=keep)
        if self.task == "segment":
            y, (feats, mc, proto) = out
            return im, y, dict(saved=saved, proto=proto, feats=feats)
        y, feats = out
        return im, y, dict(saved=saved, feats=feats)

    @torch.no_grad()
    def predict_exact(self, im: torch.Tensor, conf: float = 0.25, iou: float = 0.7, max_det: int = 300) -> List:
        """The same graph and weights evaluated in float64 (the reference's arithmetic without its
        fp32 rounding), the same NMS and clip; (n, 6) float64 rows per image.  Measures how far the fp32 reference
        itself is from the exact answer (tests/matching.py ref_f64_slack)."""
        import copy
        if getattr(self, "_net64", None) is None:
            self._net64 = copy.deepcopy(self.net).double()
        x = pp.load_tensor_check(im.float().cpu() if im.dtype != torch.float32 else im.cpu()).double()
        y, _ = self._net64(x)[0]
        shape = x.shape[2:]
        out = []
        nc = 80 if self.task == "segment" else 0
        for d in pp.non_max_suppression(y, conf, iou, None, False, max_det, nc=nc):
            d = d.clone()
            d[:, :4] = pp.scale_boxes(shape, d[:, :4], shape)
            out.append(d[:, :6])
        return out

    @torch.no_grad()
    def predict(self, im: torch.Tensor, conf: float = 0.25, iou: float = 0.7, classes: Optional[Sequence] = None,
                agnostic_nms: bool = False, max_det: int = 300) -> List[Dict]:
        im, y, ex = self.raw(im)
        nc = 80 if self.task == "segment" else 0
        dets = pp.non_max_suppression(y, conf, iou, classes, agnostic_nms, max_det, nc=nc)
        shape = im.shape[2:]
        out = []
        for b, d in enumerate(dets):
            r = {}
            if self.task == "segment":
                if len(d):
                    masks = pp.process_mask(ex["proto"][b], d[:, 6:], d[:, :4], shape, upsample=True)
                    d = d.clone()
                    d[:, :4] = pp.scale_boxes(shape, d[:, :4], shape)
                    keepm = masks.sum((-2, -1)) > 0
                    d, masks = d[keepm], masks[keepm]
                else:
                    masks = None
                r["masks"] = masks
            else:
                d = d.clone()
                d[:, :4] = pp.scale_boxes(shape, d[:, :4], shape)
            r["boxes"] = d[:, :6]
            out.append(r)
        return out
