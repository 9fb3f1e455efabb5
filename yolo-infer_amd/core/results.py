"""Results / Boxes / Masks: the per-image result objects `YOLO11Model.predict` returns.

Mirrors the subset of the Ultralytics Results contract the reference's consumers read
(/root/reference/demos/detection_demo.py:116-132 `.boxes.xyxy/.conf/.cls` per box, `.cpu().numpy()`;
/root/reference/utils/visualization.py:46-74, 370-437 `.names`, `len(boxes)`, iteration, `.masks.data`).
Tensors stay on the model's device, like upstream.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch


class _TensorView:
    def __init__(self, data):
        self.data = data

    def cpu(self):
        return self.__class__(self.data.cpu(), *self._extra()) if isinstance(self.data, torch.Tensor) else self

    def numpy(self):
        d = self.data.cpu().numpy() if isinstance(self.data, torch.Tensor) else self.data
        return self.__class__(d, *self._extra())

    def cuda(self):
        return self.__class__(torch.as_tensor(self.data).cuda(), *self._extra())

    def to(self, *args, **kwargs):
        return self.__class__(torch.as_tensor(self.data).to(*args, **kwargs), *self._extra())

    def _extra(self):
        return ()

    @property
    def shape(self):
        return self.data.shape

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.__class__(self.data[idx], *self._extra())

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class Boxes(_TensorView):
    """(n, 6) [x1, y1, x2, y2, conf, cls] detections of one image (upstream `ultralytics.engine.results.Boxes`)."""

    def __init__(self, boxes, orig_shape):
        if boxes.ndim == 1:
            boxes = boxes[None, :]
        super().__init__(boxes)
        self.orig_shape = orig_shape

    def _extra(self):
        return (self.orig_shape,)

    @property
    def xyxy(self):
        return self.data[:, :4]

    @property
    def conf(self):
        return self.data[:, 4]

    @property
    def cls(self):
        return self.data[:, 5]

    @property
    def id(self):
        return None

    @property
    def is_track(self):
        return False

    @property
    def xywh(self):
        x = self.xyxy
        y = x.clone() if isinstance(x, torch.Tensor) else np.copy(x)
        y[..., 0] = (x[..., 0] + x[..., 2]) / 2
        y[..., 1] = (x[..., 1] + x[..., 3]) / 2
        y[..., 2] = x[..., 2] - x[..., 0]
        y[..., 3] = x[..., 3] - x[..., 1]
        return y

    @property
    def xyxyn(self):
        x = self.xyxy.clone() if isinstance(self.xyxy, torch.Tensor) else np.copy(self.xyxy)
        x[..., [0, 2]] /= self.orig_shape[1]
        x[..., [1, 3]] /= self.orig_shape[0]
        return x

    @property
    def xywhn(self):
        x = self.xywh
        x[..., [0, 2]] /= self.orig_shape[1]
        x[..., [1, 3]] /= self.orig_shape[0]
        return x


class Masks(_TensorView):
    """(n, H, W) binary instance masks of one image."""

    def __init__(self, masks, orig_shape=None):
        super().__init__(masks)
        self.orig_shape = orig_shape

    def _extra(self):
        return (self.orig_shape,)


class LazyCounts:
    """The B detection counts of one asynchronous predict() call, still on the device (the words the NMS kernel
    writes behind the call's rows): read to the host once, on the first access by any of the call's Results."""

    def __init__(self, dev_counts: torch.Tensor, stream=None):
        self._dev = dev_counts
        self._host = None
        self._ev = None
        if stream is not None:  # the launch stream's point: the read may happen under another current stream
            self._ev = torch.cuda.Event()
            self._ev.record(stream)

    def __getitem__(self, b: int) -> int:
        if self._host is None:
            if self._ev is not None:
                self._ev.synchronize()
            self._host = self._dev.tolist()  # the device->host read of this call
        return self._host[b]


class Results:
    def __init__(self, orig_tensor: Optional[torch.Tensor], names: Dict[int, str], boxes: torch.Tensor,
                 masks: Optional[torch.Tensor] = None, path: str = "image0.jpg", speed=None):
        self._orig_tensor = orig_tensor
        self._orig_img = None
        self.orig_shape = tuple(orig_tensor.shape[-2:]) if orig_tensor is not None else None
        self.names = names
        self.boxes = Boxes(boxes, self.orig_shape)
        self.masks = Masks(masks, self.orig_shape) if masks is not None else None
        self.path = path
        self.speed = speed or {"preprocess": None, "inference": None, "postprocess": None}
        self.probs = None
        self.keypoints = None
        self.obb = None

    @classmethod
    def from_batch(cls, batch: torch.Tensor, b: int, names: Dict[int, str], dets: torch.Tensor, n,
                   path: str = "image0.jpg", speed=None, masks: Optional[torch.Tensor] = None,
                   moff: int = 0) -> "Results":
        """Image b of a predict() batch: boxes = dets[b, :n, :6], the input slice batch[b] and (Segment) the masks
        masks[moff : moff + n], all taken (as tensor views) on first access, so building the B Results of a call
        costs no tensor operations.  n: the count, or the call's LazyCounts (read from the device on first access)."""
        r = cls.__new__(cls)
        r._batch, r._b, r._dets, r._n = batch, b, dets, n
        r._orig_tensor_v = None
        r._orig_img = None
        r.orig_shape = tuple(batch.shape[-2:])
        r.names = names
        r._boxes = None
        r._masks = None
        r._msrc = (masks, moff) if masks is not None else None
        r.path = path
        r.speed = speed or {"preprocess": None, "inference": None, "postprocess": None}
        r.probs = r.keypoints = r.obb = None
        return r

    @classmethod
    def from_image(cls, img_bgr: np.ndarray, path: str, names: Dict[int, str], boxes: torch.Tensor,
                   masks: Optional[torch.Tensor] = None, speed=None) -> "Results":
        """An image-file / ndarray source: `orig_img` is the HWC uint8 BGR image as loaded (cv2.imread order),
        boxes are in its coordinates (already mapped back by scale_boxes)."""
        r = cls(None, names, boxes, masks=masks, path=path, speed=speed)
        r._orig_img = img_bgr
        r.orig_shape = tuple(img_bgr.shape[:2])
        r.boxes.orig_shape = r.orig_shape
        if r.masks is not None:
            r.masks.orig_shape = r.orig_shape
        return r

    @property
    def _orig_tensor(self):
        if self._orig_tensor_v is None and getattr(self, "_batch", None) is not None:
            self._orig_tensor_v = self._batch[self._b]
        return self._orig_tensor_v

    @_orig_tensor.setter
    def _orig_tensor(self, t):
        self._orig_tensor_v = t
        self._batch = None

    @property
    def _count(self) -> int:
        return self._n if isinstance(self._n, int) else self._n[self._b]

    @property
    def boxes(self) -> "Boxes":
        if self._boxes is None:
            self._boxes = Boxes(self._dets[self._b, : self._count, :6], self.orig_shape)
        return self._boxes

    @boxes.setter
    def boxes(self, b):
        self._boxes = b

    @property
    def masks(self) -> Optional["Masks"]:
        if self._masks is None and getattr(self, "_msrc", None) is not None:
            mb, moff = self._msrc
            self._masks = Masks(mb[moff:moff + self._count], self.orig_shape)
        return self._masks

    @masks.setter
    def masks(self, m):
        self._masks = m
        self._msrc = None

    @property
    def orig_img(self) -> np.ndarray:
        """HWC uint8 copy of the input image, as upstream `convert_torch2numpy_batch` makes it
        ((x.permute(1,2,0)*255).clamp(0,255).to(uint8)); materialised (one device→host copy) on first access."""
        if self._orig_img is None and self._orig_tensor is not None:
            t = self._orig_tensor
            self._orig_img = (t.permute(1, 2, 0).contiguous() * 255).clamp_(0, 255).to(torch.uint8).cpu().numpy()
        return self._orig_img

    def __len__(self):
        return len(self.boxes)

    def _like(self, orig_tensor, boxes, masks):
        r = Results(orig_tensor, self.names, boxes, masks, self.path, self.speed)
        if orig_tensor is None:  # image-file / ndarray source: keep the loaded image and its shape
            r._orig_img = self._orig_img
            r.orig_shape = self.orig_shape
            r.boxes.orig_shape = self.orig_shape
            if r.masks is not None:
                r.masks.orig_shape = self.orig_shape
        return r

    def __getitem__(self, idx):
        return self._like(self._orig_tensor, self.boxes.data[idx],
                          self.masks.data[idx] if self.masks is not None else None)

    def cpu(self):
        return self._like(self._orig_tensor.cpu() if self._orig_tensor is not None else None, self.boxes.data.cpu(),
                          self.masks.data.cpu() if self.masks is not None else None)

    def summary(self, normalize=False, decimals=5):
        out = []
        for row in self.boxes.data.tolist():
            x1, y1, x2, y2, conf, c = row[:6]
            out.append({"name": self.names[int(c)], "class": int(c), "confidence": round(conf, decimals),
                        "box": {"x1": round(x1, decimals), "y1": round(y1, decimals), "x2": round(x2, decimals),
                                "y2": round(y2, decimals)}})
        return out

    def __repr__(self):
        return f"Results(boxes={len(self.boxes)}, orig_shape={self.orig_shape})"
