"""Restated Ultralytics predict pre/post-processing (CPU, fp32). TEST INFRASTRUCTURE ONLY.

Upstream (not in /root/reference): ultralytics 8.3.x `data/loaders.py:LoadTensor._single_check`,
`utils/ops.py:{non_max_suppression, xywh2xyxy, scale_boxes, clip_boxes, process_mask, crop_mask}` and
`torchvision.ops.nms` (CPU kernel `nms_kernel_impl`).  Call sites in the reference: `core/model.py:133`
(predict), `demos/detection_demo.py:87-93,116-132` (Results consumer).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn.functional as F


def load_tensor_check(im: torch.Tensor, stride: int = 32) -> torch.Tensor:
    """LoadTensor._single_check: BCHW (3-D is unsqueezed), H,W % 32 == 0, /255 if max > 1 + eps(dtype)."""
    if im.dim() != 4:
        if im.dim() != 3:
            raise ValueError("torch.Tensor inputs should be BCHW")
        im = im.unsqueeze(0)
    if im.shape[2] % stride or im.shape[3] % stride:
        raise ValueError(f"torch.Tensor inputs should be divisible by stride {stride}")
    if im.max() > 1.0 + torch.finfo(im.dtype).eps:
        im = im.float() / 255.0
    return im


def xywh2xyxy(x: torch.Tensor) -> torch.Tensor:
    y = torch.empty_like(x)
    xy = x[..., :2]
    wh = x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def nms_greedy(boxes: torch.Tensor, scores: torch.Tensor, iou_thres: float) -> torch.Tensor:
    """torchvision.ops.nms (CPU kernel): stable descending sort, greedy, suppress IoU > thr, no +1 in areas."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.long)
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    order = scores.sort(stable=True, descending=True)[1]
    n = boxes.shape[0]
    x1l, y1l, x2l, y2l, al = (t.tolist() for t in (x1, y1, x2, y2, areas))
    ordl = order.tolist()
    sup = [False] * n
    keep = []
    f32 = torch.float32
    for _i in range(n):
        i = ordl[_i]
        if sup[i]:
            continue
        keep.append(i)
        # vectorised over the remaining boxes, fp32 arithmetic exactly as the C++ loop does it
        rest = order[_i + 1:]
        if rest.numel() == 0:
            continue
        xx1 = torch.clamp(x1[rest], min=x1l[i])
        yy1 = torch.clamp(y1[rest], min=y1l[i])
        xx2 = torch.clamp(x2[rest], max=x2l[i])
        yy2 = torch.clamp(y2[rest], max=y2l[i])
        w = torch.clamp(xx2 - xx1, min=0.0)
        h = torch.clamp(yy2 - yy1, min=0.0)
        inter = w * h
        ovr = inter / ((torch.tensor(al[i], dtype=f32) + areas[rest]) - inter)
        hit = (ovr.double() > iou_thres).tolist()
        for j, hflag in zip(rest.tolist(), hit):
            if hflag:
                sup[j] = True
    return torch.tensor(keep, dtype=torch.long)


def non_max_suppression(prediction: torch.Tensor, conf_thres=0.25, iou_thres=0.45, classes: Optional[Sequence] = None,
                        agnostic=False, max_det=300, nc=0, max_nms=30000, max_wh=7680) -> List[torch.Tensor]:
    """ops.non_max_suppression (single-label path, no time limit: it never triggers on the oracle sizes)."""
    bs = prediction.shape[0]
    nc = nc or (prediction.shape[1] - 4)
    extra = prediction.shape[1] - nc - 4
    mi = 4 + nc
    xc = prediction[:, 4:mi].amax(1) > conf_thres
    prediction = prediction.transpose(-1, -2)
    prediction = torch.cat((xywh2xyxy(prediction[..., :4]), prediction[..., 4:]), dim=-1)
    cls_t = torch.tensor(classes) if classes is not None else None
    output = [torch.zeros((0, 6 + extra))] * bs
    for xi, x in enumerate(prediction):
        x = x[xc[xi]]
        if not x.shape[0]:
            continue
        box, cls, mask = x.split((4, nc, extra), 1)
        conf, j = cls.max(1, keepdim=True)
        x = torch.cat((box, conf, j.float(), mask), 1)[conf.view(-1) > conf_thres]
        if cls_t is not None:
            x = x[(x[:, 5:6] == cls_t).any(1)]
        n = x.shape[0]
        if not n:
            continue
        if n > max_nms:
            x = x[x[:, 4].argsort(descending=True)[:max_nms]]
        c = x[:, 5:6] * (0 if agnostic else max_wh)
        i = nms_greedy(x[:, :4] + c, x[:, 4], iou_thres)
        output[xi] = x[i[:max_det]]
    return output


def clip_boxes(boxes: torch.Tensor, shape) -> torch.Tensor:
    boxes[..., 0] = boxes[..., 0].clamp(0, shape[1])
    boxes[..., 1] = boxes[..., 1].clamp(0, shape[0])
    boxes[..., 2] = boxes[..., 2].clamp(0, shape[1])
    boxes[..., 3] = boxes[..., 3].clamp(0, shape[0])
    return boxes


def scale_boxes(img1_shape, boxes, img0_shape, padding=True):
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    pad = (round((img1_shape[1] - img0_shape[1] * gain) / 2 - 0.1),
           round((img1_shape[0] - img0_shape[0] * gain) / 2 - 0.1))
    if padding:
        boxes[..., 0] -= pad[0]
        boxes[..., 1] -= pad[1]
        boxes[..., 2] -= pad[0]
        boxes[..., 3] -= pad[1]
    boxes[..., :4] /= gain
    return clip_boxes(boxes, img0_shape)


def crop_mask(masks, boxes):
    _, h, w = masks.shape
    x1, y1, x2, y2 = torch.chunk(boxes[:, :, None], 4, 1)
    r = torch.arange(w, dtype=x1.dtype)[None, None, :]
    c = torch.arange(h, dtype=x1.dtype)[None, :, None]
    return masks * ((r >= x1) * (r < x2) * (c >= y1) * (c < y2))


def process_mask(protos, masks_in, bboxes, shape, upsample=False):
    c, mh, mw = protos.shape
    ih, iw = shape
    masks = (masks_in @ protos.float().view(c, -1)).view(-1, mh, mw)
    db = bboxes.clone()
    db[:, 0] *= mw / iw
    db[:, 2] *= mw / iw
    db[:, 3] *= mh / ih
    db[:, 1] *= mh / ih
    masks = crop_mask(masks, db)
    if upsample:
        masks = F.interpolate(masks[None], shape, mode="bilinear", align_corners=False)[0]
    return masks.gt_(0.0)
