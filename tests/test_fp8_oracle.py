"""CPU tests of the fp8 (e4m3) PTQ variant: the oracle's restatement (oracle/quant.py backend "fp8"), the product's
fp8 packing (yolomi.quant / yolomi.plan dtype "f8") and the committed fp8 fixture.

BASELINE config 4 reads "yolo11n PTQ int8 ... fp8 MFMA"; SURVEY §8(c) asks for e4m3 vectors emulated with
torch.float8_e4m3fn.  The reference's own qconfig (/root/reference/optimization/quantization/quantizers.py:124-131)
is int8 only, so the fp8 plan is this build's variant of it: the same quantisation points, e4m3 codes with
amax / 448 scales.  Parity of the fp8 GPU plan with this oracle is a tolerance (tests/test_gpu_fp8.py).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import quant as Q
from tests.golden.make_golden import F8_FIXTURES, make_input
from tests.matching import MatchReport, match_image
from yolomi.arch import GraphBuilder
from yolomi.synth import synth_weights

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def e4m3_reference(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even onto the e4m3 grid, written out from the format (1-4-3, bias 7, max 448, subnormal
    step 2^-9), independently of torch's cast: the value closest to x, ties to the even significand."""
    x = np.asarray(x, np.float64)
    out = np.empty_like(x)
    for i, v in np.ndenumerate(x):
        a = min(abs(v), 448.0)
        if a < 2.0 ** -6:  # subnormal range: multiples of 2^-9
            step = 2.0 ** -9
        else:
            e = int(np.floor(np.log2(a)))
            step = 2.0 ** (e - 3)
        q = a / step
        f = np.floor(q)
        r = q - f
        n = f + (1 if (r > 0.5 or (r == 0.5 and int(f) % 2 == 1)) else 0)
        out[i] = np.copysign(min(n * step, 448.0), v)
    return out


def test_fp8_quantize_is_rne_onto_the_e4m3_grid():
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.standard_normal(4000) * 50, rng.standard_normal(2000) * 0.01,
                        np.array([0.0, -0.0, 448.0, 449.0, 464.0, 1e6, -1e6, 2.0 ** -10, 3 * 2.0 ** -10, 2.0 ** -9,
                                  1.0625, 1.1875, 17.0, 19.0, -17.0])]).astype(np.float32)
    got = Q.quantize_fp8(torch.from_numpy(v), 1.0).numpy()
    assert np.array_equal(got, e4m3_reference(v).astype(np.float32))
    assert np.isfinite(got).all() and np.abs(got).max() == 448.0


def test_product_fp8_weights_equal_the_oracle():
    """yolomi.quant.quantize_weight_fp8 (codes for the GPU blob) decodes to exactly the oracle's e4m3 weights."""
    from yolomi.plan import _conv_weights
    from yolomi.quant import e4m3_table, quantize_weight_fp8
    sd = synth_weights("n", "detect", 0)
    mods = dict(Q.build_folded("n", "detect", sd).named_modules())
    g = GraphBuilder("n", "detect", quant=True)
    ops = {op.name: op for op in g.ops}
    tab = e4m3_table()
    for p in ("model.0", "model.2.m.0.cv2", "model.9.cv2", "model.23.cv2.0.2", "model.23.cv3.0.0.1"):
        w, _ = _conv_weights(ops[p].args, sd)
        conv = mods[p].conv if hasattr(mods[p], "conv") else mods[p]
        codes, s1 = quantize_weight_fp8(w)
        v2, s2 = Q.quantize_weight_fp8(conv.weight)
        assert np.array_equal(s1, s2), p
        assert np.array_equal(np.transpose(tab[codes], (0, 3, 1, 2)), v2.numpy()), p


def test_fp8_post_table_is_the_oracle_activation():
    from yolomi.quant import e4m3_table, post_table_fp8
    s = 0.0371
    tab = e4m3_table()
    ok = np.isfinite(torch.arange(256).to(torch.uint8).view(torch.float8_e4m3fn).float().numpy())
    x = torch.from_numpy(tab[ok]) * Q._t32(s)
    assert np.array_equal(post_table_fp8(s, True)[ok], Q.silu64(x).numpy())
    assert np.array_equal(post_table_fp8(s, False)[ok], x.numpy())


def test_fp8_blob_packs_and_rejects_int8_qparams():
    from yolomi.plan import DTYPES, pack_model
    sd = synth_weights("n", "detect", 0)
    net = Q.build_folded("n", "detect", sd)
    qp = Q.calibrate(net, [make_input("uniform", (3,), 64)], "fp8")
    assert all(v[1] == 0 for k, v in qp.items() if k != "backend")
    blob = pack_model("n", "detect", sd, "f8", qp)
    assert np.frombuffer(blob[:12], np.int32)[2] == DTYPES["f8"]
    with pytest.raises(ValueError):
        pack_model("n", "detect", sd, "f8", Q.calibrate(net, [make_input("uniform", (3,), 64)], "qnnpack"))
    with pytest.raises(ValueError):
        pack_model("n", "detect", sd, "i8", qp)


@pytest.mark.parametrize("name", list(F8_FIXTURES))
def test_fp8_oracle_reproduces_golden(name):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    sd = synth_weights(g["scale"], "detect", 0)
    net = Q.build_folded(g["scale"], "detect", sd)
    qp = Q.calibrate(net, [make_input("uniform", tuple(g["calibration"]["seeds"]), g["calibration"]["size"])], "fp8")
    assert Q.qparams_to_json(qp) == g["qparams"]
    m = Q.Int8OracleModel(g["scale"], "detect", sd, Q.qparams_from_json(g["qparams"]))
    res = m.predict(make_input("uniform", tuple(g["input"]["seeds"]), g["input"]["size"]), conf=g["conf"], iou=g["iou"])
    rep = MatchReport()
    for r, got in zip(g["dets"], res):
        match_image(np.array(r, np.float32).reshape(-1, 6), got["boxes"].numpy(), g["conf"], g["iou"], 1e-4, 1e-5,
                    rep=rep)
    assert rep.ok and rep.matched == sum(len(d) for d in g["dets"]), str(rep)
