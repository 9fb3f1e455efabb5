"""Restated Ultralytics predict preprocessing for image sources. TEST INFRASTRUCTURE ONLY.

Upstream (not in /root/reference): ultralytics 8.3.x
  * `engine/predictor.py:BasePredictor.preprocess / pre_transform`: a list of HWC BGR uint8 images (cv2.imread order)
    is letterboxed with `LetterBox(imgsz, auto=same_shapes and model.pt, stride=32)`, stacked, `[..., ::-1]` (BGR ->
    RGB), transposed to BCHW, `.float() / 255`;
  * `data/augment.py:LetterBox.__call__` (center=True, scaleup=True, padding value 114);
  * `cv2.resize(img, new_unpad, interpolation=cv2.INTER_LINEAR)` for 8-bit images: OpenCV's fixed-point bilinear
    (imgproc/src/resize.cpp: 11-bit coefficients, `HResizeLinear` then `VResizeLinear` with `FixedPtCast<.., 22>`);
  * `utils/ops.py:scale_boxes` maps detections back (oracle/postprocess.py).
Call sites in the reference: `demos/detection_demo.py:87-93, 190-196` (path / ndarray sources of predict()).

Parity with cv2 itself is UNPINNED: OpenCV is not installed here and its 8-bit linear resize has three
implementations that can differ by one level on some pixels (the scalar fixed-point path restated below, the SIMD
path's `(S >> 4) * b >> 16` rounding, and IPP in the opencv-python wheels).  This restatement is the scalar path;
the GPU kernel (csrc/ym_letterbox.hip) reproduces it bit for bit.  The letterbox geometry (sizes, padding split,
stride rounding) is exact Ultralytics arithmetic.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS  # INTER_RESIZE_COEF_SCALE


def letterbox_geometry(h: int, w: int, new_shape=(640, 640), auto=True, stride=32, scaleup=True) -> Tuple:
    """LetterBox.__call__ arithmetic: returns (unpad_h, unpad_w, top, bottom, left, right)."""
    r = min(new_shape[0] / h, new_shape[1] / w)
    if not scaleup:
        r = min(r, 1.0)
    new_unpad = int(round(w * r)), int(round(h * r))  # (w, h); Python round = half to even, as upstream
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, stride), np.mod(dh, stride)
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return new_unpad[1], new_unpad[0], top, bottom, left, right


def _axis(src: int, dst: int):
    """Per destination index: source index pair and 11-bit weights (resize.cpp, INTER_LINEAR coefficient setup:
    fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), clamped at both borders with fx = 0; each weight
    saturate_cast<short>(w * 2048), i.e. rounded to nearest even)."""
    scale = 1.0 / (dst / src)  # scale_x = 1. / inv_scale_x, inv_scale_x = (double)dst / src
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    hi = s >= src - 1
    f[hi], s[hi] = 0, src - 1
    a0 = np.rint((np.float32(1) - f) * np.float32(COEF_SCALE)).astype(np.int64)
    a1 = np.rint(f * np.float32(COEF_SCALE)).astype(np.int64)
    s1 = np.minimum(s + 1, src - 1)
    return s, s1, a0, a1, hi


def resize_linear_u8(img: np.ndarray, new_h: int, new_w: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation=cv2.INTER_LINEAR) for HWC uint8, scalar fixed-point path:
    horizontal sums S = src[sx]·a0 + src[sx+1]·a1 (right border: src[sx]·2048), then
    dst = (S(row sy)·b0 + S(row sy+1)·b1 + 2^21) >> 22, saturated to [0, 255]."""
    h, w = img.shape[:2]
    if (h, w) == (new_h, new_w):
        return img.copy()
    sx, sx1, a0, a1, xhi = _axis(w, new_w)
    sy, sy1, b0, b1, _ = _axis(h, new_h)
    src = img.astype(np.int64)
    hs = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]
    hs[:, xhi, :] = src[:, sx[xhi], :] * COEF_SCALE  # the right border uses one sample
    v = hs[sy] * b0[:, None, None] + hs[sy1] * b1[:, None, None]
    return np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def letterbox(img: np.ndarray, new_shape=(640, 640), auto=True, stride=32) -> np.ndarray:
    """LetterBox()(image=img) for one HWC BGR uint8 image: resize (if the shape changes), pad with 114."""
    h, w = img.shape[:2]
    uh, uw, top, bottom, left, right = letterbox_geometry(h, w, new_shape, auto, stride)
    if (h, w) != (uh, uw):
        img = resize_linear_u8(img, uh, uw)
    out = np.full((uh + top + bottom, uw + left + right, img.shape[2]), 114, np.uint8)
    out[top:top + uh, left:left + uw] = img
    return out


def preprocess(images: Sequence[np.ndarray], imgsz: int = 640, stride: int = 32) -> np.ndarray:
    """BasePredictor.preprocess for a list of HWC BGR uint8 images: (B, 3, H, W) float32 RGB in [0, 1]."""
    same = len({im.shape for im in images}) == 1
    lb = [letterbox(im, (imgsz, imgsz), auto=same, stride=stride) for im in images]
    x = np.stack(lb)[..., ::-1].transpose(0, 3, 1, 2)
    return np.ascontiguousarray(x).astype(np.float32) / np.float32(255)


def batch_geometry(shapes: List[Tuple[int, int]], imgsz: int = 640, stride: int = 32) -> Tuple[int, int]:
    """Letterboxed (H, W) of a batch of (h, w) image shapes (auto only when all shapes agree)."""
    same = len(set(shapes)) == 1
    h, w = shapes[0]
    uh, uw, top, bottom, left, right = letterbox_geometry(h, w, (imgsz, imgsz), auto=same, stride=stride)
    return uh + top + bottom, uw + left + right
