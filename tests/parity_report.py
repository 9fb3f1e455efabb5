"""Layer-by-layer parity report: HIP engine buffers vs the CPU oracle (run on a GPU box).

    python tests/parity_report.py --scale n --dtype f32 --batch 2

Prints, for every plan buffer that corresponds to an oracle layer output (`L{i}`) plus the anchor-major head
buffer, the max abs / relative error, then the detection match report (tests/matching.py).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

from oracle.predict import OracleModel  # noqa: E402
from tests.matching import match_image, MatchReport  # noqa: E402
from yolomi.engine import Engine  # noqa: E402
from yolomi.synth import synth_weights, uniform  # noqa: E402


def make_input(B, H, W, seed=1234, kind="uniform"):
    x = uniform(seed, B * 3 * H * W).astype(np.float32).reshape(B, 3, H, W)
    if kind == "randn":
        from yolomi.synth import normal
        x = normal(seed, B * 3 * H * W).astype(np.float32).reshape(B, 3, H, W)
    return torch.from_numpy(x)


def report(scale="n", task="detect", dtype="f32", B=2, H=640, W=640, seed=0, kind="uniform", verbose=True):
    sd = synth_weights(scale, task, seed)
    om = OracleModel(scale, task, sd)
    x = make_input(B, H, W, kind=kind)
    im, y, ex = om.raw(x, keep=tuple(range(23)))
    eng = Engine(scale, task, sd, torch.device("cuda", 0), dtype)
    xg = x.cuda()
    t = time.time()
    dets, counts = eng.run(xg, use_graph=False)
    torch.cuda.synchronize()
    if verbose:
        print(f"[{scale} {dtype} B={B}] eager forward {1e3 * (time.time() - t):.1f} ms (first call)")
    worst = 0.0
    rows = []
    for b in eng.graph.buffers:
        if b.name.startswith("L") and b.name[1:].isdigit():
            i = int(b.name[1:])
            ref = ex["saved"][i].permute(0, 2, 3, 1).contiguous()
            got = eng.read_buffer(b.id, B)
            err = (got - ref).abs().max().item()
            rel = err / max(ref.abs().max().item(), 1e-6)
            worst = max(worst, rel)
            rows.append((b.name, tuple(ref.shape), err, rel))
    # head: anchor-major (B, A, no)
    feats = ex["feats"]
    no = eng.graph.no
    ref_h = torch.cat([f.view(B, no, -1) for f in feats], 2).transpose(1, 2)
    got_h = eng.read_buffer(eng.graph.anchor_buf.id, B).reshape(B, -1, eng.graph.anchor_buf.C)[..., :no]
    herr = (got_h - ref_h).abs().max().item()
    rows.append(("head", tuple(ref_h.shape), herr, herr / max(ref_h.abs().max().item(), 1e-6)))
    if verbose:
        for r in rows:
            print(f"  {r[0]:>6} {str(r[1]):>22} max|d|={r[2]:.3e} rel={r[3]:.3e}")
    # detections
    ref_dets = om.predict(x)
    n = counts.cpu().tolist()
    got_dets = dets.cpu().numpy()
    tol_xy = 1e-3 if dtype == "f32" else 1e-3 * max(H, W)
    tol_s = 1e-3
    rep = MatchReport()
    for bi in range(B):
        match_image(ref_dets[bi]["boxes"].numpy(), got_dets[bi, : n[bi], :6], 0.25, 0.7, tol_xy, tol_s, rep=rep)
    if verbose:
        print(f"  dets: build {n} oracle {[len(d['boxes']) for d in ref_dets]} :: {rep}")
        for f in rep.failures[:5]:
            print("   ", f)
    return rows, rep, eng, x


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", default="n")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--kind", default="uniform")
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    report(a.scale, a.task, a.dtype, a.batch, a.size, a.size, kind=a.kind)
