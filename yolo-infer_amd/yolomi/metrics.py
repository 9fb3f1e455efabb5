"""Offline detection metrics: mAP50 / mAP50-95.

Semantics of the numbers the reference reads from Ultralytics val (`core/validator.py:339-352`:
`results.box.map`, `.map50`, `.map75`, `.mp`, `.mr`): per class, predictions sorted by confidence, a prediction is
a TP at IoU threshold t as upstream `BaseValidator.match_predictions` decides it (ultralytics 8.3.x,
engine/validator.py); AP = area under the 101-point COCO-interpolated precision envelope; mAP = mean over classes
present in the ground truth, mAP50-95 = mean over t ∈ {0.50, 0.55, ..., 0.95}.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

IOUV = np.linspace(0.5, 0.95, 10)


def box_iou(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:4], b[None, :, 2:4])
    inter = np.clip(rb - lt, 0, None).prod(2)
    aa = (a[:, 2:4] - a[:, :2]).prod(1)
    ab = (b[:, 2:4] - b[:, :2]).prod(1)
    return inter / np.maximum(aa[:, None] + ab[None] - inter, 1e-9)


def match_predictions(pred: np.ndarray, gt: np.ndarray) -> np.ndarray:
    """pred (n,6) [xyxy,conf,cls] in NMS (confidence-descending) order, gt (m,6) [xyxy,-,cls] → TP (n, 10) bool.

    Upstream's non-scipy branch: the (gt, pred) pairs with IoU >= t and equal class, sorted by IoU descending; keep
    each prediction's best pair (np.unique on the prediction index, which leaves the pairs in prediction-index
    order); then each ground truth keeps its FIRST remaining pair in that order — the lowest prediction index, i.e.
    the most confident prediction, not the highest IoU (upstream's re-sort by IoU between the two steps is commented
    out).  Equal IoUs: upstream's `argsort()[::-1]` leaves their order to numpy's quicksort; here it is stable."""
    tp = np.zeros((len(pred), len(IOUV)), bool)
    if len(pred) == 0 or len(gt) == 0:
        return tp
    iou = box_iou(gt[:, :4], pred[:, :4])
    iou = iou * (gt[:, None, 5] == pred[None, :, 5])
    for k, t in enumerate(IOUV):
        m = np.argwhere(iou >= t)
        if len(m):
            if len(m) > 1:
                v = iou[m[:, 0], m[:, 1]]
                m = m[np.argsort(-v, kind="stable")]
                m = m[np.unique(m[:, 1], return_index=True)[1]]
                m = m[np.unique(m[:, 0], return_index=True)[1]]
            tp[m[:, 1], k] = True
    return tp


def compute_ap(recall: np.ndarray, precision: np.ndarray) -> float:
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    y = np.interp(x, mrec, mpre)
    return float(((y[1:] + y[:-1]) / 2 * np.diff(x)).sum())


def evaluate(preds: List[np.ndarray], gts: List[np.ndarray]) -> Dict[str, float]:
    """preds/gts: per-image (n,6) arrays [x1,y1,x2,y2,conf,cls] (gt conf ignored). Returns map50, map75, map."""
    tps, confs, pcls, gcls = [], [], [], []
    for p, g in zip(preds, gts):
        p = np.asarray(p, np.float64).reshape(-1, 6)
        g = np.asarray(g, np.float64).reshape(-1, 6)
        tps.append(match_predictions(p, g))
        confs.append(p[:, 4])
        pcls.append(p[:, 5])
        gcls.append(g[:, 5])
    tp = np.concatenate(tps) if tps else np.zeros((0, 10), bool)
    conf = np.concatenate(confs) if confs else np.zeros(0)
    pc = np.concatenate(pcls) if pcls else np.zeros(0)
    gc = np.concatenate(gcls) if gcls else np.zeros(0)
    order = np.argsort(-conf, kind="stable")
    tp, pc = tp[order], pc[order]
    classes = np.unique(gc)
    ap = np.zeros((len(classes), len(IOUV)))
    for ci, c in enumerate(classes):
        sel = pc == c
        n_gt = int((gc == c).sum())
        if sel.sum() == 0 or n_gt == 0:
            continue
        fpc = (1 - tp[sel]).cumsum(0)
        tpc = tp[sel].cumsum(0)
        recall = tpc / (n_gt + 1e-16)
        precision = tpc / (tpc + fpc)
        for k in range(len(IOUV)):
            ap[ci, k] = compute_ap(recall[:, k], precision[:, k])
    if len(classes) == 0:
        return {"map50": 0.0, "map75": 0.0, "map": 0.0}
    return {"map50": float(ap[:, 0].mean()), "map75": float(ap[:, 5].mean()), "map": float(ap.mean())}
