"""GPU parity of the x3 plan (fp32 activations, every conv GEMM as three split-f16 MFMAs: csrc/ym_conv.hip mma<x3_t>).

The benched plan, held to the north-star bar (BASELINE.json: "within 1e-3 on coords/scores and exact on class
indices" against the reference's fp32 CPU path, /root/reference/core/model.py:133), which the plain f16 plan misses
by ~600x on coordinates.  Tolerance written here:
  * every oracle detection matched or exempt (tests/matching.py) — no min_frac —
    with |Δscore| <= 5e-5, class exact, and |Δxy| <= 1e-3 px ABSOLUTE beyond the fp32 oracle's own rounding error
    for that detection: the bound per row is 1e-3 + |oracle_fp32 − oracle_float64| (tests/matching.py ref_f64_slack;
    the same graph evaluated in float64, oracle/predict.py predict_exact).  The fp32 reference arithmetic itself sits
    up to 7-8e-4 px from the float64 answer on yolo11s (tools/x3_emulate.py), so two faithful fp32 evaluations of one
    graph can differ by > 1e-3 px on the largest stride-32 boxes; a dropped split term (~2^-11 relative: 0.3-0.6 px)
    still fails by two orders of magnitude;
  * and, tighter than that slack (triangle inequality), the GPU's own distance from the float64 answer: the same
    matching protocol (and exemptions) with the float64 evaluation as the reference, at TOL_EXACT_XY = 5e-4 px and
    5e-5 score;
  * per-layer outputs within 1e-4 relative of the oracle.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.predict import OracleModel
from tests.golden.make_golden import make_input
from tests.matching import MatchReport, match_image, ref_f64_slack
from yolomi.synth import synth_weights

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = torch.device("cuda", 0)
TOL_XY, TOL_S = 1e-3, 5e-5  # the north-star bar (px absolute, score)
TOL_EXACT_XY = 5e-4  # the GPU's own distance from the float64 evaluation of the same graph (px), per detection
_cache = {}


def oracle(scale="n", task="detect"):
    k = ("o", scale, task)
    if k not in _cache:
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        _cache[k] = OracleModel(scale, task, synth_weights(scale, task, 0))
    return _cache[k]


def model(scale="n", task="detect", fuse_dw=True):
    """fuse_dw=False: the plan with the Detect-head depthwise convs as their own ops (YM_FUSE_DW=0), whose cv3
    1x1 → 1x1 pairs then run on the streaming kernel's x3 FUSE mode."""
    from core.model import YOLO11Model
    k = ("m", scale, task, fuse_dw)
    if k not in _cache:
        if not fuse_dw:
            os.environ["YM_FUSE_DW"] = "0"
        try:
            _cache[k] = YOLO11Model(task=task, size=scale, device="cuda:0", dtype="x3", verbose=False)
        finally:
            os.environ.pop("YM_FUSE_DW", None)
    return _cache[k]


def check(ref_dets, got_results, conf=0.25, iou=0.7, max_det=300, x=None, scale="n", task="detect"):
    """x (the CPU input): the per-row bound takes the oracle's own fp32 error from a float64 evaluation, and the
    GPU's own distance from that float64 answer is held to TOL_EXACT_XY / TOL_S directly."""
    rep, rex = MatchReport(), MatchReport()
    exact = oracle(scale, task).predict_exact(x, conf, iou, max_det) if x is not None else None
    for b, (r, g) in enumerate(zip(ref_dets, got_results)):
        ref = r["boxes"].numpy() if isinstance(r, dict) else np.asarray(r, np.float32).reshape(-1, 6)
        got = g.boxes.data.cpu().numpy()
        tol = ref_f64_slack(ref, exact[b].numpy(), TOL_XY) if exact is not None else TOL_XY
        match_image(ref, got, conf, iou, tol, TOL_S, rep=rep, max_det=max_det)
        if exact is not None:  # the same protocol (and exemptions) against the float64 evaluation, at the exact bar
            match_image(exact[b].numpy(), got.astype(np.float64), conf, iou, TOL_EXACT_XY, TOL_S, rep=rex,
                        max_det=max_det)
    print(f"x3 parity: {rep}; GPU vs float64: {rex}")
    assert rep.ok, f"{rep}; {rep.failures[:3]}"
    assert rep.matched > 0
    if exact is not None:
        assert rex.ok and rex.matched > 0, f"GPU vs float64: {rex}; {rex.failures[:3]}"
    return rep


def _rel(got, ref):
    return (got - ref).abs().max().item() / ref.abs().max().item()


def test_x3_layers_match_oracle():
    eng = model("n").model.engine
    x = make_input("uniform", (11, 12), 640)
    _, y, ex = oracle().raw(x, keep=(2, 4, 6, 8, 9, 10, 13, 16, 19, 22))
    eng.run(x.to(DEV), use_graph=False)
    for b in eng.graph.buffers:
        if b.name.startswith("L") and b.name[1:].isdigit() and int(b.name[1:]) in ex["saved"]:
            ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
            assert _rel(eng.read_buffer(b.id, 2), ref) < 1e-4, b.name
    no = eng.graph.no
    ref_h = torch.cat([f.view(2, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
    got_h = eng.read_buffer(eng.graph.anchor_buf.id, 2).reshape(2, -1, eng.graph.anchor_buf.C)[..., :no]
    assert _rel(got_h, ref_h) < 1e-4


@pytest.mark.parametrize("name", ["det_n_uniform", "det_n_randn", "det_n_320_lowconf", "det_s_uniform"])
def test_x3_plan_matches_golden(name):
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    x = make_input(g["input"]["kind"], g["input"]["seeds"], g["input"]["size"])
    res = model(g["scale"]).predict(x.to(DEV), conf=g["conf"], iou=g["iou"])
    check(g["dets"], res, g["conf"], g["iou"], x=x, scale=g["scale"])


@pytest.mark.parametrize("scale", ["n", "s"])
def test_x3_b8_matches_oracle(scale):
    """BASELINE configs 2 and 3 (B=8, 640x640) under the tile table the bench runs, at the SURVEY f16 tolerance."""
    x = make_input("uniform", tuple(range(7001, 7009)), 640)
    ref = oracle(scale).predict(x)
    m = model(scale)
    res = m.predict(x.to(DEV))
    rep = check(ref, res, x=x, scale=scale)
    assert rep.max_dscore <= TOL_S


@pytest.mark.parametrize("conf", [0.05, 0.004])
def test_x3_low_conf(conf):
    """Thousands of candidates per image (every NMS path) at the f16-mode tolerance."""
    x = make_input("uniform", (31, 32), 640)
    check(oracle().predict(x, conf=conf), model("n").predict(x.to(DEV), conf=conf), conf=conf, x=x)


def test_x3_segment_s_b4():
    """BASELINE config 5 (yolo11s-seg, B=4): boxes, the 32 mask coefficients of every match, and masks."""
    g = json.load(open(os.path.join(GOLD, "seg_s_uniform.json")))
    x = make_input("uniform", g["input"]["seeds"], 640)
    m = model("s", "segment")
    eng = m.model.engine
    dets, counts = eng.run(x.to(DEV), conf=g["conf"], iou=g["iou"])
    rep, rex, worst = MatchReport(), MatchReport(), 0.0
    exact = oracle("s", "segment").predict_exact(x, g["conf"], g["iou"])
    for b, n in enumerate(counts.tolist()):
        r = np.asarray(g["nms_rows"][b], np.float32).reshape(-1, 38)
        got = dets[b, :int(n)].cpu().numpy()
        before = len(rep.pairs)
        match_image(r[:, :6], got[:, :6], g["conf"], g["iou"], ref_f64_slack(r[:, :6], exact[b].numpy(), TOL_XY),
                    TOL_S, rep=rep)
        scale = max(float(np.abs(r[:, 6:]).max()) if len(r) else 1.0, 1e-6)
        for i, j in rep.pairs[before:]:
            worst = max(worst, float(np.abs(r[i, 6:] - got[j, 6:]).max()) / scale)
        match_image(exact[b].numpy(), got[:, :6].astype(np.float64), g["conf"], g["iou"], TOL_EXACT_XY, TOL_S, rep=rex)
    print(f"x3 segment parity: {rep}, mask coefficients {worst:.3g} of max; GPU vs float64: {rex}")
    assert rep.ok and rep.matched > 0, rep
    assert rex.ok and rex.matched > 0, f"GPU vs float64: {rex}; {rex.failures[:3]}"
    assert worst <= 1e-3, worst
    ref = oracle("s", "segment").predict(x, conf=0.25)
    res = m.predict(x.to(DEV), conf=0.25)
    for r, gg in zip(ref, res):
        rb, gb = r["boxes"].numpy(), gg.boxes.data.cpu().numpy()
        assert len(rb) == len(gb)
        for i in np.argsort(-rb[:, 4]):
            j = int(np.argmin(np.abs(gb[:, :4] - rb[i, :4]).max(1)))
            a = (r["masks"][i] == gg.masks.data[j].cpu()).float().mean().item()
            assert a >= 0.999, (i, j, a)


# csrc/ym_conv.hip: 12 direct-to-register + 5 LDS-staged tile configurations, then the 30 LDS-DMA ones
# (csrc/ym_conv_dma.hip) and 31 streaming ones (csrc/ym_conv_stream.hip), x3 pairing mode; then the 9 x3-only LDS-DMA
# split-K ones (after the 116-id f16 catalogue).
X3_CFGS = list(range(17)) + list(range(17, 47)) + list(range(47, 78)) + list(range(116, 125))


@pytest.mark.parametrize("cfg", X3_CFGS)
def test_x3_conv_configs_match_oracle(cfg):
    """Every x3 conv kernel configuration on every conv of yolo11n (1x1 two-source / up-sampled, 3x3 s1/s2,
    residual epilogues, fp32 Detect rows; ops a configuration does not take fall back to the heuristic tile): layer
    outputs within 1e-4 of the oracle."""
    eng = model("n").model.engine
    x = make_input("uniform", (11, 12), 640)
    _, y, ex = oracle().raw(x, keep=(2, 4, 6, 8, 9, 10, 13, 16, 19, 22))
    xd = x.to(DEV)
    try:
        eng.run(xd, use_graph=False)
        eng.rt.set_op_cfg(2, 640, 640, [cfg if op.kind == "conv" else -1 for op in eng.graph.ops])
        eng.run(xd, use_graph=False)
        for b in eng.graph.buffers:
            if b.name.startswith("L") and b.name[1:].isdigit() and int(b.name[1:]) in ex["saved"]:
                ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
                assert _rel(eng.read_buffer(b.id, 2), ref) < 1e-4, (cfg, b.name)
    finally:
        eng._tuned.discard((2, 640, 640))


def test_x3_1280_n1600_attention_and_max_nms():
    """x3 at 1280² (N = 1600: the block-wise x3 MFMA attention) and conf 0.001 (> max_nms candidates): every
    detection within the SURVEY f16-mode tolerance, and the attention layer within 1e-4 of the oracle."""
    x = make_input("uniform", (8101,), 1280)
    _, y, ex = oracle().raw(x, keep=(10,))
    eng = model("n").model.engine
    eng.run(x.to(DEV), use_graph=False)
    b = [b for b in eng.graph.buffers if b.name == "L10"][0]
    assert _rel(eng.read_buffer(b.id, 1), ex["saved"][10].permute(0, 2, 3, 1)) < 1e-4
    assert int((y[0, 4:84].amax(0) > 0.001).sum()) > 30000
    check(oracle().predict(x, conf=0.001), model("n").predict(x.to(DEV), conf=0.001), conf=0.001, x=x)


SPLIT_TAG = 1 << 20  # csrc/ym_runtime.cpp kSplitTag: op cfg of a fused pair run as its two convs
STREAM_BASE, N_STREAM = 17 + 30, 31  # csrc/ym_conv.hip: first-gen + LDS-DMA ids, then the streaming kernels
BNECK_BASE, N_BNECK = 17 + 30 + 43 + 12, 14  # ... + streaming/small-M + halo ids, then the fused Bottleneck kernels
X3_BNECK = (116 + 9, 116 + 11)  # x3-only ids: after the f16 catalogue and the 9 x3-only LDS-DMA configurations


@pytest.mark.parametrize("scale", ["n", "s"])
def test_x3_fused_pairs_match_split(scale):
    """x3 fused pairs against the same plan with its pairs run as two launches, Detect rows within 2e-6 relative (the
    same split products summed in another order; the plan's own per-layer parity is test_x3_layers_match_oracle):
      * conv -> 1x1 pairs (csrc/ym_conv_stream.hip FUSE in the x3 mode: the intermediate split hi/lo in registers,
        three 16x16x16 MFMAs per K block of the second GEMM) on every streaming configuration, and on the LDS-DMA
        kernel's fused-epilogue GEMM (csrc/ym_conv_dma.hip FUSE: the intermediate split into the idle stage ring);
      * Bottlenecks (csrc/ym_conv_bneck.hip in the x3 mode: hi / lo LDS planes, three MFMAs per K step) on every
        tile variant, the x3-only 2 x 32 tiles included (the ones whose doubled LDS does not fit fall back to the
        split pair).
    (On the plan without the depthwise fusion: with it the head's cv3 1x1s are depthwise-fused, not paired.)"""
    eng = model(scale, fuse_dw=False).model.engine
    x = make_input("uniform", (21, 22), 640).to(DEV)
    B, _, H, W = x.shape
    ops = eng.graph.ops
    pairs = [i for i, op in enumerate(ops) if op.args.get("pair")]
    bneck = [i for i in pairs if ops[i].args["pair"]["k"] == 3]
    assert len(pairs) - len(bneck) >= 4 and len(bneck) >= 2
    eng.run(x, use_graph=False)
    tuned = eng.rt.get_op_cfg(B, H, W)
    base = [c if op.kind == "conv" and not op.args.get("pair") else -1 for c, op in zip(tuned, ops)]
    try:
        split = list(base)
        for i in pairs:
            split[i] = SPLIT_TAG + 256 * 29 + 29  # one LDS-DMA tile for both convs (inapplicable: the heuristic)
        eng.rt.set_op_cfg(B, H, W, split)
        eng.run(x, use_graph=False)
        ref = eng.read_buffer(eng.graph.anchor_buf.id, B)
        band = list(range(BNECK_BASE, BNECK_BASE + N_BNECK)) + list(range(*X3_BNECK))
        # conv -> 1x1 pairs: the streaming FUSE mode, the LDS-DMA kernel's fused-epilogue GEMM (DMA ids 17..46, those
        # of YM_DMA_FUSE_CFGS instantiated) and the band kernel's x3 stride-2 "down" mode (model.1+cv1: the tiles
        # whose doubled LDS fits)
        dma = list(range(17, 17 + 30))
        for cfgs, ids in ((list(range(STREAM_BASE, STREAM_BASE + N_STREAM)) + dma + band,
                           [i for i in pairs if i not in bneck]),
                          (band, bneck)):
            for c in cfgs:
                cfg = list(split)
                for i in ids:
                    cfg[i] = c
                eng.rt.set_op_cfg(B, H, W, cfg)
                eng.run(x, use_graph=False)
                got = eng.read_buffer(eng.graph.anchor_buf.id, B)
                assert _rel(got, ref) < 2e-6, c
    finally:
        eng.rt.set_op_cfg(B, H, W, tuned)


def test_x3_pair_stores_bitwise_equal():
    """The lane-pair epilogue stores (csrc/ym_common.h ym_p2_store4_pair; family mask YM_DBG_PAIRST, read at graph
    capture) write the same bits as the per-lane stores: yolo11s B=8 under the committed x3 table with every family's
    pairing off (0), on with the ds_bpermute exchange (15) and on with the v_permlane*_swap exchange (31) — the
    detection rows of all eight images are bitwise equal."""
    from core.model import YOLO11Model
    from yolomi import lib as L
    x = make_input("uniform", list(range(8)), 640).to(DEV)
    rows = {}
    prev = L.set_debug(L.DBG_PAIRST, 0)
    try:
        for mask in ("0", "15", "31"):
            L.set_debug(L.DBG_PAIRST, int(mask) + 1)
            m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
            rows[mask] = [r.boxes.data.clone() for r in m.predict(x, conf=0.05)]
            del m
    finally:
        L.set_debug(L.DBG_PAIRST, prev)
    assert sum(len(r) for r in rows["0"]) > 100
    for mask in ("15", "31"):
        for a, b in zip(rows["0"], rows[mask]):
            assert a.shape == b.shape and torch.equal(a, b), f"YM_PAIRST={mask}: detections differ from the per-lane stores"


def test_x3_literal_bar_on_the_bench_batch():
    """The literal north-star bar (BASELINE.json: 1e-3 on coordinates and scores, class exact, against the fp32 CPU
    oracle — no float64 slack) on the very batch `bench.py` times and reports (`synthetic_batch(8, 640, 1000)`,
    yolo11s x3 under the committed B=8 table), through bench.py's own `parity()`.  The bar is met on this batch
    (8.7e-4 px) but not on every batch, since the fp32 oracle is itself up to 8e-4 px from float64: this
    test gates the figure the bench line reports, so a table or kernel change that moves it past 1e-3 fails here."""
    import bench
    from core.model import YOLO11Model
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    x = bench.synthetic_batch(8, 640, 1000, DEV)
    m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
    gdets = [r.boxes.data.cpu().numpy() for r in m.predict(x)]
    om = OracleModel("s", "detect", synth_weights("s", "detect", 0))
    gts = [r["boxes"].numpy() for r in om.predict(x.cpu())]
    p = bench.parity(gdets, gts)
    assert p["matched"] > 100 and p["meets_tolerance"], p
