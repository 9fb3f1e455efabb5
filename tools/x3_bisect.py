#!/usr/bin/env python3
"""Where the x3 plan's coordinate error comes from: the GPU's layer outputs injected into a float64 forward.

For checkpoint layer k, every layer output the rest of the graph reads from layers <= k is taken from the GPU
(read back from the plan's buffers after one eager x3 forward), and layers k+1 .. Detect + decode + NMS run in
float64 on the CPU.  The detections' distance from the all-float64 answer is then the error the GPU's layers <= k
contribute.  Checkpoint 23 = the GPU's raw Detect rows decoded in float64 (only the decode is exact); "gpu" = the
GPU's own detections (its fp32 decode included).

    python tools/x3_bisect.py [s] [8] [seed]

Runs on the GPU box (bench batch: bench.synthetic_batch(B, 640, 1000 + rank) with rank 0).  Test infrastructure:
imports oracle/ as the checker.
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import postprocess as pp  # noqa: E402
from oracle.predict import OracleModel  # noqa: E402
from tests.matching import iou_matrix  # noqa: E402

FROMS = {12: (-1, 6), 15: (-1, 4), 18: (-1, 13), 21: (-1, 10), 23: (16, 19, 22)}


def needed_after(k, n_layers=24):
    """Layer outputs (<= k) that layers > k read."""
    need = {k}
    for i in range(k + 1, n_layers):
        for j in FROMS.get(i, ()):
            if j != -1 and j <= k:
                need.add(j)
    return need


@torch.no_grad()
def forward_from(net64, k, inj):
    """Layers k+1.. of the oracle's module list in float64, with y[j] = inj[j] for the injected outputs."""
    y = [None] * len(net64.model)
    for j, t in inj.items():
        y[j] = t
    x = y[k]
    for i in range(k + 1, len(net64.model)):
        m = net64.model[i]
        if i in FROMS:
            x = [x if j == -1 else y[j] for j in FROMS[i]]
        x = m(x)
        y[i] = x
    return x[0] if isinstance(x, tuple) else x


def dets_of(y, conf=0.25, iou=0.7, shape=(640, 640)):
    """NMS then the clip of predict()'s scale_boxes (oracle/predict.py), as predict_exact."""
    out = []
    for d in pp.non_max_suppression(y.double(), conf, iou, None, False, 300):
        d = d.clone()
        d[:, :4] = pp.scale_boxes(shape, d[:, :4], shape)
        out.append(d[:, :6].numpy())
    return out


def dist_to(exact, got):
    """max over got's detections of the coordinate distance to the same-class float64 detection (IoU >= 0.99)."""
    worst, n, miss = 0.0, 0, 0
    for e, g in zip(exact, got):
        if not len(g):
            continue
        ious = iou_matrix(g[:, :4], e[:, :4]) if len(e) else np.zeros((len(g), 0))
        for i in range(len(g)):
            c = np.where((e[:, 5] == g[i, 5]) & (ious[i] >= 0.99))[0] if len(e) else []
            if not len(c):
                miss += 1
                continue
            worst = max(worst, float(np.abs(e[c, :4] - g[i, :4]).max(1).min()))
            n += 1
    return worst, n, miss


def main():
    from bench import synthetic_batch
    from core.model import YOLO11Model
    from yolomi.synth import synth_weights
    scale = sys.argv[1] if len(sys.argv) > 1 else "s"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    torch.set_num_threads(16)
    dev = torch.device("cuda", 0)
    x = synthetic_batch(B, 640, seed, dev)
    m = YOLO11Model(task="detect", size=scale, device="cuda:0", dtype="x3", verbose=False)
    res = m.predict(x)
    gpu = [r.boxes.data.cpu().numpy().astype(np.float64) for r in res]
    eng = m.model.engine
    eng.run(x, use_graph=False)
    bufs = {b.name: b for b in eng.graph.buffers}

    om = OracleModel(scale, "detect", synth_weights(scale, "detect", 0))
    net64 = copy.deepcopy(om.net).double()
    xc = x.cpu()
    y32 = om.raw(xc)[1]
    with torch.no_grad():
        (y64, _), _ = net64(xc.double())
    exact = dets_of(y64)
    print(f"yolo11{scale} x3 B={B} seed {seed}: {sum(len(e) for e in exact)} float64 detections", flush=True)
    w, n, miss = dist_to(exact, dets_of(y32))
    print(f"  fp32 oracle            max|dxy| vs float64 {w:.3e} px  ({n} matched, {miss} unmatched)", flush=True)
    w, n, miss = dist_to(exact, gpu)
    print(f"  GPU detections         max|dxy| vs float64 {w:.3e} px  ({n} matched, {miss} unmatched)", flush=True)
    for k in (2, 4, 6, 8, 9, 10, 13, 16, 19, 22):
        inj = {}
        for j in needed_after(k):
            t = eng.read_buffer(bufs[f"L{j}"].id, B)  # NHWC fp32 (hi + lo)
            inj[j] = t.permute(0, 3, 1, 2).contiguous().double()
        y = forward_from(net64, k, inj)
        w, n, miss = dist_to(exact, dets_of(y))
        print(f"  GPU layers <= {k:2d}, rest float64: max|dxy| {w:.3e} px  ({n} matched, {miss} unmatched)", flush=True)
    # the GPU's raw Detect rows (anchor-major (B, A, no)) decoded in float64
    det = net64.model[23]
    no = det.no
    rows = eng.read_buffer(eng.graph.anchor_buf.id, B)
    rows = rows.reshape(B, -1, rows.shape[-1])[..., :no].double()
    feats, a0 = [], 0
    for s in (8, 16, 32):
        h = w_ = 640 // s
        feats.append(rows[:, a0:a0 + h * w_].transpose(1, 2).reshape(B, no, h, w_))
        a0 += h * w_
    with torch.no_grad():
        y = det._inference(feats)
    w, n, miss = dist_to(exact, dets_of(y))
    print(f"  GPU Detect rows, float64 decode:  max|dxy| {w:.3e} px  ({n} matched, {miss} unmatched)", flush=True)
    # per detection: which stride level carries the worst GPU error
    worst = []
    for e, g in zip(exact, gpu):
        if not len(g) or not len(e):
            continue
        ious = iou_matrix(g[:, :4], e[:, :4])
        for i in range(len(g)):
            c = np.where((e[:, 5] == g[i, 5]) & (ious[i] >= 0.99))[0]
            if len(c):
                d = float(np.abs(e[c, :4] - g[i, :4]).max(1).min())
                wh = float(max(g[i, 2] - g[i, 0], g[i, 3] - g[i, 1]))
                worst.append((d, wh))
    worst.sort(reverse=True)
    print("  worst GPU detections (|dxy| px, box size px):", [(round(a, 6), round(b, 1)) for a, b in worst[:8]])


if __name__ == "__main__":
    main()
