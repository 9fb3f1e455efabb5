"""Detection matching protocol for parity.

Per image: for each oracle detection (score-descending) find an unmatched build detection of the SAME class with
IoU >= 0.99 and require |Δcoord| <= tol_xy, |Δscore| <= tol_score.  Oracle detections whose score is within
`conf_margin` of the confidence threshold, or that sit in an NMS near-tie (another same-class oracle box with IoU
within `iou_margin` of the NMS threshold), are EXEMPT: an ulp-level difference can legitimately flip them.
Build detections left unmatched are checked the same way against the exemption rules from the build side.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import numpy as np


def iou_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    x1 = np.maximum(a[:, None, 0], b[None, :, 0])
    y1 = np.maximum(a[:, None, 1], b[None, :, 1])
    x2 = np.minimum(a[:, None, 2], b[None, :, 2])
    y2 = np.minimum(a[:, None, 3], b[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / np.maximum(aa[:, None] + ab[None, :] - inter, 1e-12)


@dataclass
class MatchReport:
    matched: int = 0
    exempt: int = 0
    unmatched_ref: int = 0
    unmatched_build: int = 0
    max_dxy: float = 0.0
    max_dscore: float = 0.0
    failures: List[str] = field(default_factory=list)
    pairs: List[tuple] = field(default_factory=list)  # (ref row, build row) of every match, in the callers' order

    @property
    def ok(self) -> bool:
        return self.unmatched_ref == 0 and self.unmatched_build == 0

    def __str__(self):
        return (f"matched={self.matched} exempt={self.exempt} unmatched_ref={self.unmatched_ref} "
                f"unmatched_build={self.unmatched_build} max|dxy|={self.max_dxy:.3g} "
                f"max|dscore|={self.max_dscore:.3g}")


def _exempt(d: np.ndarray, same: np.ndarray, conf: float, iou_thr: float, conf_margin: float,
            iou_margin: float) -> np.ndarray:
    ex = np.abs(d[:, 4] - conf) <= conf_margin
    if len(d):
        m = iou_matrix(d[:, :4], same[:, :4]) if len(same) else np.zeros((len(d), 0))
        if m.size:
            cls_eq = d[:, None, 5] == same[None, :, 5]
            near = (np.abs(m - iou_thr) <= iou_margin) & cls_eq
            ex |= near.any(1)
    return ex


def match_image(ref: np.ndarray, got: np.ndarray, conf: float, iou_thr: float, tol_xy, tol_score: float,
                conf_margin: float = 2e-3, iou_margin: float = 1e-3, rep: MatchReport = None,
                max_det: int = 300) -> MatchReport:
    """When a list is truncated at max_det, detections scoring within conf_margin of the last kept score are
    exempt too (which of several near-equal candidates make the cut is an ulp-level decision).  iou_margin is
    SURVEY §8(c)'s 1e-3.  tol_xy: one bound, or one per reference row (in `ref`'s order; ref_f64_slack)."""
    rep = rep or MatchReport()
    tol_row = np.broadcast_to(np.asarray(tol_xy, np.float64), (len(ref),))
    oref = np.argsort(-ref[:, 4], kind="stable") if len(ref) else np.zeros(0, np.int64)
    ogot = np.argsort(-got[:, 4], kind="stable") if len(got) else np.zeros(0, np.int64)
    ref = ref[oref] if len(ref) else ref.reshape(0, ref.shape[1] if ref.ndim == 2 else 6)
    got = got[ogot] if len(got) else got.reshape(0, got.shape[1] if got.ndim == 2 else 6)
    cut = -np.inf
    for d in (ref, got):
        if len(d) >= max_det:
            cut = max(cut, float(d[:, 4].min()))
    used = np.zeros(len(got), bool)
    ious = iou_matrix(ref[:, :4], got[:, :4])

    def exempt(d, same):
        if not len(d):
            return np.zeros(0, bool)
        ex = _exempt(d, same, conf, iou_thr, conf_margin, iou_margin)
        return ex | (d[:, 4] <= cut + conf_margin)

    ex_ref = exempt(ref, ref)
    for i in range(len(ref)):
        cand = np.where((~used) & (got[:, 5] == ref[i, 5]) & (ious[i] >= 0.99))[0] if len(got) else []
        ok = False
        for j in cand:
            dxy = float(np.abs(got[j, :4] - ref[i, :4]).max())
            ds = float(abs(got[j, 4] - ref[i, 4]))
            if dxy <= tol_row[oref[i]] and ds <= tol_score:
                used[j] = True
                rep.matched += 1
                rep.pairs.append((int(oref[i]), int(ogot[j])))
                rep.max_dxy = max(rep.max_dxy, dxy)
                rep.max_dscore = max(rep.max_dscore, ds)
                ok = True
                break
        if not ok:
            if ex_ref[i]:
                rep.exempt += 1
            else:
                rep.unmatched_ref += 1
                rep.failures.append(f"ref det {ref[i].tolist()} unmatched")
    rest = got[~used]
    if len(rest):
        ex_b = exempt(rest, got)
        rep.exempt += int(ex_b.sum())
        rep.unmatched_build += int((~ex_b).sum())
        for r in rest[~ex_b]:
            rep.failures.append(f"build det {r.tolist()} unmatched")
    return rep


def ref_f64_slack(ref: np.ndarray, exact: np.ndarray, tol_xy: float = 1e-3) -> np.ndarray:
    """Per-row coordinate bound for matching against an fp32 reference `ref` whose own rounding error is known:
    tol_xy plus that row's distance from the same detection computed in float64 (`exact`: the reference graph run in
    float64, same NMS; matched by class and IoU >= 0.99; a row with no float64 counterpart keeps tol_xy).  The bar
    then reads "within tol_xy of the reference, beyond the reference's own fp32 rounding": on yolo11s the fp32 path
    itself sits up to 8e-4 px from the float64 answer (tools/x3_emulate.py), so two faithful fp32 evaluations of the
    same graph can differ by more than 1e-3 px on the largest stride-32 boxes."""
    out = np.full(len(ref), tol_xy, np.float64)
    if not len(ref) or not len(exact):
        return out
    ious = iou_matrix(ref[:, :4], exact[:, :4])
    for i in range(len(ref)):
        cand = np.where((exact[:, 5] == ref[i, 5]) & (ious[i] >= 0.99))[0]
        if len(cand):
            out[i] = tol_xy + float(np.abs(exact[cand, :4] - ref[i, :4]).max(1).min())
    return out

