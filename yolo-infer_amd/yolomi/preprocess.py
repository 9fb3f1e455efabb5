"""Image sources for predict(): decoding, Ultralytics LetterBox geometry, and the GPU letterbox.

Ultralytics 8.3.x `BasePredictor.pre_transform` letterboxes a list of HWC BGR uint8 images (cv2.imread order) with
`LetterBox(imgsz, auto=same_shapes, stride=32)` (auto: the canvas shrinks to the stride multiple when every image
has the same shape, else every image goes to imgsz x imgsz), stacks them, flips BGR→RGB, moves to the device and
divides by 255.  Here the geometry is computed on the host (`letterbox_geometry`, the same arithmetic as
`LetterBox.__call__`), each image is copied to the device once, and `ym_letterbox` (csrc/ym_letterbox.hip) writes
its slot of the fp32 NCHW batch.  Detections are mapped back with `scale_boxes` (upstream `ops.scale_boxes`).
Reference call sites: /root/reference/demos/detection_demo.py:87-93, 190-196 (path / ndarray sources).
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np
import torch

IMG_SUFFIXES = {".bmp", ".dng", ".jpeg", ".jpg", ".mpo", ".png", ".tif", ".tiff", ".webp", ".pfm", ".heic"}


def letterbox_geometry(h: int, w: int, new_shape=(640, 640), auto=True, stride=32, scaleup=True) -> Tuple:
    """LetterBox.__call__: (unpad_h, unpad_w, top, bottom, left, right) for an h x w image."""
    r = min(new_shape[0] / h, new_shape[1] / w)
    if not scaleup:
        r = min(r, 1.0)
    uw, uh = int(round(w * r)), int(round(h * r))
    dw, dh = new_shape[1] - uw, new_shape[0] - uh
    if auto:
        dw, dh = dw % stride, dh % stride
    dw, dh = dw / 2, dh / 2
    return uh, uw, int(round(dh - 0.1)), int(round(dh + 0.1)), int(round(dw - 0.1)), int(round(dw + 0.1))


def load_image(path: str) -> np.ndarray:
    """HWC uint8 BGR array of an image file (cv2.imread order; decoded with Pillow, which this image ships)."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


def expand_sources(source) -> Tuple[List[np.ndarray], List[str]]:
    """predict() sources other than tensors → (list of HWC uint8 BGR arrays, list of paths)."""
    items = list(source) if isinstance(source, (list, tuple)) else [source]
    imgs, paths = [], []
    for i, s in enumerate(items):
        if isinstance(s, (str, os.PathLike)):
            p = os.fspath(s)
            if os.path.isdir(p):
                files = sorted(f for f in os.listdir(p) if os.path.splitext(f)[1].lower() in IMG_SUFFIXES)
                for f in files:
                    imgs.append(load_image(os.path.join(p, f)))
                    paths.append(os.path.join(p, f))
                continue
            if not os.path.exists(p):
                raise FileNotFoundError(f"{p} does not exist")
            imgs.append(load_image(p))
            paths.append(p)
        elif isinstance(s, np.ndarray):
            if s.ndim == 2:
                s = np.repeat(s[..., None], 3, axis=2)
            if s.ndim != 3 or s.shape[2] != 3 or s.dtype != np.uint8:
                raise ValueError(f"ndarray sources must be HWC uint8 with 3 channels (BGR), got {s.shape} {s.dtype}")
            imgs.append(np.ascontiguousarray(s))
            paths.append(f"image{i}.jpg")
        elif hasattr(s, "convert") and hasattr(s, "size"):  # PIL.Image
            rgb = np.asarray(s.convert("RGB"))
            imgs.append(np.ascontiguousarray(rgb[..., ::-1]))
            paths.append(getattr(s, "filename", "") or f"image{i}.jpg")
        else:
            raise TypeError(f"unsupported source type {type(s).__name__}")
    if not imgs:
        raise FileNotFoundError("no images found in source")
    return imgs, paths


def letterbox_batch(rt, imgs: Sequence[np.ndarray], device: torch.device, imgsz: int = 640, stride: int = 32,
                    stream: int = 0) -> Tuple[torch.Tensor, List[Tuple[int, int]]]:
    """The predictor's preprocessed batch (B, 3, Hn, Wn) fp32 on `device`, built on the GPU."""
    same = len({im.shape for im in imgs}) == 1
    geo = [letterbox_geometry(im.shape[0], im.shape[1], (imgsz, imgsz), auto=same, stride=stride) for im in imgs]
    uh, uw, t, b, l, r = geo[0]
    Hn, Wn = uh + t + b, uw + l + r
    out = torch.empty((len(imgs), 3, Hn, Wn), dtype=torch.float32, device=device)
    srcs = [torch.from_numpy(im).to(device, non_blocking=False) for im in imgs]
    for i, (im, g) in enumerate(zip(srcs, geo)):
        h, w = im.shape[:2]
        rt.letterbox(im.data_ptr(), h, w, im.stride(0), True, g[0], g[1], g[2], g[4], out[i].data_ptr(), Hn, Wn,
                     stream)
    return out, [im.shape[:2] for im in imgs]


def scale_boxes(img1_shape, boxes: torch.Tensor, img0_shape) -> torch.Tensor:
    """ops.scale_boxes(img1_shape, boxes, img0_shape) (padding=True) + clip_boxes, in place on an (n, >=4) tensor."""
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
           round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    boxes[..., 0] -= pad[0]
    boxes[..., 1] -= pad[1]
    boxes[..., 2] -= pad[0]
    boxes[..., 3] -= pad[1]
    boxes[..., :4] /= gain
    boxes[..., 0].clamp_(0, img0_shape[1])
    boxes[..., 1].clamp_(0, img0_shape[0])
    boxes[..., 2].clamp_(0, img0_shape[1])
    boxes[..., 3].clamp_(0, img0_shape[0])
    return boxes
