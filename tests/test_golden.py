"""The CPU oracle reproduces the committed golden fixtures (tests/golden/make_golden.py).  Pins the oracle +
portable synthetic weights across hosts/torch builds; the GPU path is checked against the same fixtures in
tests/test_gpu_parity.py.  (Parity with Ultralytics itself is unpinned: see oracle/__init__.py.)"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.predict import OracleModel
from tests.golden.make_golden import LAYERS, make_input
from tests.matching import MatchReport, match_image
from yolomi.synth import synth_weights

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return json.load(open(os.path.join(GOLD, name + ".json")))


@pytest.mark.parametrize("name", ["det_n_uniform", "det_n_randn", "det_n_320_lowconf"])
def test_oracle_reproduces_golden(name):
    g = load(name)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    om = OracleModel(g["scale"], "detect", synth_weights(g["scale"], "detect", g["weights_seed"]))
    x = make_input(g["input"]["kind"], g["input"]["seeds"], g["input"]["size"])
    im, y, ex = om.raw(x, keep=LAYERS)
    for i in LAYERS:
        t = ex["saved"][i].permute(0, 2, 3, 1).double()
        ref = g["layers"][f"L{i}"]
        assert list(t.shape) == ref["shape"]
        assert float(t.abs().sum()) == pytest.approx(ref["abs_sum"], rel=1e-5)
        np.testing.assert_allclose(t.reshape(-1)[ref["samples_idx"]].numpy(), ref["samples"], rtol=1e-4, atol=1e-5)
    dets = om.predict(x, conf=g["conf"], iou=g["iou"])
    rep = MatchReport()
    for d, r in zip(dets, g["dets"]):
        match_image(np.array(r, np.float32).reshape(-1, 6), d["boxes"].numpy(), g["conf"], g["iou"], 1e-3, 1e-4,
                    rep=rep)
    assert rep.ok, rep.failures[:3]
    assert rep.matched >= 0.9 * sum(len(r) for r in g["dets"])


def test_golden_files_are_small_and_complete():
    total = sum(os.path.getsize(os.path.join(GOLD, f)) for f in os.listdir(GOLD))
    assert total < 2_000_000
    for name in ("det_n_uniform", "det_n_randn", "det_n_320_lowconf", "det_s_uniform", "seg_s_uniform"):
        g = load(name)
        assert len(g["dets"]) == len(g["input"]["seeds"]) and all(len(d) > 0 for d in g["dets"])


def test_oracle_reproduces_segment_golden():
    """yolo11s-seg B=4 (BASELINE config 5): NMS rows incl. the 32 mask coefficients, proto, and per-mask extents."""
    from oracle import postprocess as pp
    g = load("seg_s_uniform")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    om = OracleModel("s", "segment", synth_weights("s", "segment", 0))
    x = make_input("uniform", g["input"]["seeds"], 640)
    im, y, ex = om.raw(x)
    t = ex["proto"].permute(0, 2, 3, 1).double()
    assert float(t.abs().sum()) == pytest.approx(g["proto"]["abs_sum"], rel=1e-5)
    np.testing.assert_allclose(t.reshape(-1)[g["proto"]["samples_idx"]].numpy(), g["proto"]["samples"], rtol=1e-4,
                               atol=1e-5)
    nms = pp.non_max_suppression(y, g["conf"], g["iou"], nc=80)
    for d, rows in zip(nms, g["nms_rows"]):
        d = d.clone()
        d[:, :4] = pp.clip_boxes(d[:, :4], (640, 640))
        r = torch.tensor(rows)
        assert d.shape == r.shape
        np.testing.assert_allclose(d.numpy(), r.numpy(), rtol=1e-4, atol=1e-4)
    res = om.predict(x, conf=g["conf"], iou=g["iou"])
    for rr, ms in zip(res, g["masks"]):
        got = [[int(k.sum())] for k in rr["masks"].to(torch.int64)]
        assert len(got) == len(ms)
        for a, b in zip(got, ms):
            assert abs(a[0] - b[0]) <= max(2, 1e-3 * b[0])
