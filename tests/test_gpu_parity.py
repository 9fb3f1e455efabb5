"""GPU parity tests (MI355X): the HIP path through the C-ABI vs the CPU oracle and the golden fixtures.

Tolerances (north_star: 1e-3 on coords/scores, exact class indices):
  * f32 plan (exact-f32 MFMA, the parity mode): every matched detection |Δxy| <= 1e-3 px, |Δscore| <= 1e-3, same
    class; per-layer relative error <= 1e-4.
  * f16 plan (the throughput mode, fp16 storage + fp32 accumulation): per-layer relative error <= 1e-2;
    detections |Δxy| <= 1 px, |Δscore| <= 1e-2; >= 90 % of oracle detections matched (an NMS near-tie flip
    cascades under fp16 storage).
Exemptions follow tests/matching.py (score within 2e-3 of conf, NMS near-ties within SURVEY §8(c)'s 1e-3 of `iou`,
max_det cut-off).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.predict import OracleModel
from tests.golden.make_golden import make_input
from tests.matching import MatchReport, match_image
from yolomi.synth import synth_weights

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = torch.device("cuda", 0)

_cache = {}


def oracle(scale="n", task="detect"):
    k = ("o", scale, task)
    if k not in _cache:
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        _cache[k] = OracleModel(scale, task, synth_weights(scale, task, 0))
    return _cache[k]


def model(scale="n", dtype="f32", task="detect"):
    from core.model import YOLO11Model
    k = ("m", scale, dtype, task)
    if k not in _cache:
        _cache[k] = YOLO11Model(task=task, size=scale, device="cuda:0", dtype=dtype)
    return _cache[k]


def check(ref_dets, got_results, conf, iou, tol_xy, tol_s, min_frac=1.0, max_det=300):
    rep = MatchReport()
    for r, g in zip(ref_dets, got_results):
        ref = r["boxes"].numpy() if isinstance(r, dict) else np.asarray(r, np.float32).reshape(-1, 6)
        match_image(ref, g.boxes.data.cpu().numpy(), conf, iou, tol_xy, tol_s, rep=rep, max_det=max_det)
    total = sum(len(r["boxes"]) if isinstance(r, dict) else len(r) for r in ref_dets)
    if min_frac >= 1.0:
        assert rep.ok, f"{rep}; {rep.failures[:3]}"
    else:
        assert rep.matched + rep.exempt >= min_frac * total, f"{rep}; {rep.failures[:3]}"
    return rep


# ------------------------------------------------------------------------------------------------ layer bisect
@pytest.mark.parametrize("dtype,tol", [("f32", 1e-4), ("f16", 1e-2)])
def test_layers_match_oracle(dtype, tol):
    m = model("n", dtype)
    eng = m.model.engine
    x = make_input("uniform", (11, 12), 640)
    _, y, ex = oracle().raw(x, keep=(2, 4, 6, 8, 9, 10, 13, 16, 19, 22))
    eng.run(x.to(DEV), use_graph=False)
    for b in eng.graph.buffers:
        if b.name.startswith("L") and b.name[1:].isdigit() and int(b.name[1:]) in ex["saved"]:
            ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
            got = eng.read_buffer(b.id, 2)
            rel = (got - ref).abs().max().item() / ref.abs().max().item()
            assert rel < tol, (b.name, rel)
    no = eng.graph.no
    ref_h = torch.cat([f.view(2, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
    got_h = eng.read_buffer(eng.graph.anchor_buf.id, 2).reshape(2, -1, eng.graph.anchor_buf.C)[..., :no]
    assert (got_h - ref_h).abs().max().item() / ref_h.abs().max().item() < tol


# ------------------------------------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", ["det_n_uniform", "det_n_randn", "det_n_320_lowconf", "det_s_uniform"])
def test_f32_plan_matches_golden(name):
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    x = make_input(g["input"]["kind"], g["input"]["seeds"], g["input"]["size"]).to(DEV)
    res = model(g["scale"], "f32").predict(x, conf=g["conf"], iou=g["iou"])
    check(g["dets"], res, g["conf"], g["iou"], 1e-3, 1e-3)


@pytest.mark.parametrize("name", ["det_n_uniform", "det_s_uniform"])
def test_f16_plan_matches_golden(name):
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    x = make_input(g["input"]["kind"], g["input"]["seeds"], g["input"]["size"]).to(DEV)
    res = model(g["scale"], "f16").predict(x, conf=g["conf"], iou=g["iou"])
    check(g["dets"], res, g["conf"], g["iou"], 1.0, 1e-2, min_frac=0.9)


# ------------------------------------------------------------------------------------------------ predict kwargs
@pytest.mark.parametrize("kw", [dict(conf=0.1), dict(conf=0.25, iou=0.45), dict(conf=0.05, max_det=7),
                                dict(conf=0.1, agnostic_nms=True), dict(conf=0.1, classes=[0, 17, 42, 79])])
def test_predict_kwargs_f32(kw):
    x = make_input("uniform", (21,), 640)
    ref = oracle().predict(x, conf=kw.get("conf", 0.25), iou=kw.get("iou", 0.7), classes=kw.get("classes"),
                           agnostic_nms=kw.get("agnostic_nms", False), max_det=kw.get("max_det", 300))
    res = model("n", "f32").predict(x.to(DEV), **kw)
    check(ref, res, kw.get("conf", 0.25), kw.get("iou", 0.7), 1e-3, 1e-3, max_det=kw.get("max_det", 300))
    if "classes" in kw:
        assert set(res[0].boxes.cls.cpu().int().tolist()) <= set(kw["classes"])
    if "max_det" in kw:
        assert len(res[0]) <= kw["max_det"]


@pytest.mark.parametrize("conf", [0.5, 0.3, 0.15, 0.06, 0.02, 0.004, 0.001])
def test_nms_paths_f32(conf):
    """Candidate counts from a few dozen to thousands per image: the one-wave (<= 64), bit-matrix (<= 512) and
    blocked (> 512; the validator's conf 0.001) NMS paths of csrc/ym_misc.hip nms_image all reproduce torchvision's
    greedy order."""
    x = make_input("uniform", (31, 32), 640)
    ref = oracle().predict(x, conf=conf)
    res = model("n", "f32").predict(x.to(DEV), conf=conf)
    check(ref, res, conf, 0.7, 1e-3, 1e-3)


@pytest.mark.parametrize("S,B", [(320, 3), (1280, 1), (640, 8)])
def test_sizes_and_batches_f32(S, B):
    x = make_input("uniform", tuple(range(31, 31 + B)), S)
    ref = oracle().predict(x, conf=0.25)
    res = model("n", "f32").predict(x.to(DEV), conf=0.25)
    assert len(res) == B
    check(ref, res, 0.25, 0.7, 1e-3, 1e-3)


def test_non_square_and_empty():
    x = make_input("uniform", (41,), 640)[:, :, :384, :]  # 384 x 640
    x = x.contiguous()
    ref = oracle().predict(x, conf=0.25)
    res = model("n", "f32").predict(x.to(DEV), conf=0.25)
    check(ref, res, 0.25, 0.7, 1e-3, 1e-3)
    none = model("n", "f32").predict(x.to(DEV), conf=0.999)  # no candidate survives
    assert len(none[0]) == 0 and none[0].boxes.xyxy.shape == (0, 4)


def test_chw_input_and_cpu_tensor_source():
    x = make_input("uniform", (51,), 320)
    r1 = model("n", "f32").predict(x[0], conf=0.2)  # CHW on the CPU: unsqueezed and moved, as LoadTensor does
    r2 = model("n", "f32").predict(x.to(DEV), conf=0.2)
    assert torch.equal(r1[0].boxes.data, r2[0].boxes.data)


def test_graph_replay_bitwise_equals_eager():
    eng = model("n", "f16").model.engine
    x = make_input("uniform", (61, 62), 640).to(DEV)
    d1, c1 = eng.run(x, use_graph=False)
    d1, c1 = d1.clone(), c1.clone()
    for _ in range(3):
        d2, c2 = eng.run(x, use_graph=True)
    assert torch.equal(c1, c2) and torch.equal(d1, d2)


@pytest.mark.parametrize("dtype,scale", [("f16", "n"), ("f16", "s"), ("f32", "n")])
def test_branch_schedule_bitwise_equals_serial(dtype, scale):
    """The one-lane branch schedule (csrc/ym_runtime.cpp build_schedule: Detect-head chains on their own streams
    beside the neck) computes exactly what the serial launch order computes: same kernels, so bit-equal outputs."""
    from core.model import YOLO11Model
    x = make_input("uniform", tuple(range(41, 49)), 640).to(DEV)
    os.environ["YM_BRANCHES"] = "1"  # the serial launch order
    try:
        m = YOLO11Model(size=scale, device="cuda:0", dtype=dtype, verbose=False)
    finally:
        del os.environ["YM_BRANCHES"]
    eng = m.model.engine
    d1, c1 = eng.run(x, use_graph=True)
    d1, c1 = d1.clone(), c1.clone()
    h1 = eng.read_buffer(eng.graph.anchor_buf.id, 8)
    os.environ["YM_BRANCHES"] = "4"
    try:
        ms = YOLO11Model(size=scale, device="cuda:0", dtype=dtype, verbose=False)
    finally:
        del os.environ["YM_BRANCHES"]
    es = ms.model.engine
    for use_graph in (False, True):
        d2, c2 = es.run(x, use_graph=use_graph)
        assert torch.equal(c1, c2), use_graph
        for b, n in enumerate(c1.tolist()):  # rows past the count are whatever an earlier call left there
            assert torch.equal(d1[b, :n], d2[b, :n]), (use_graph, b)
    assert torch.equal(h1, es.read_buffer(es.graph.anchor_buf.id, 8))


# ------------------------------------------------------------------------------------------------ image sources
LB_SHAPES = [(853, 1280), (480, 640), (100, 37), (640, 640), (1000, 700)]


def _images(shapes, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in shapes]


@pytest.mark.parametrize("shapes", [[s] for s in LB_SHAPES] + [LB_SHAPES[:3], [(853, 1280)] * 3])
def test_letterbox_kernel_matches_oracle(shapes):
    """csrc/ym_letterbox.hip (fixed-point INTER_LINEAR, 114 border, BGR->RGB, /255) == oracle/letterbox.py, bit for
    bit, for single images, mixed-shape batches (auto=False: 640x640 canvases) and same-shape batches (auto=True)."""
    from oracle import letterbox as olb
    from yolomi.preprocess import letterbox_batch
    imgs = _images(shapes, 17)
    eng = model("n", "f32").model.engine
    got, _ = letterbox_batch(eng.rt, imgs, DEV, stream=torch.cuda.current_stream().cuda_stream)
    ref = torch.from_numpy(olb.preprocess(imgs))
    assert got.shape == ref.shape and torch.equal(got.cpu(), ref)


def test_predict_image_sources_match_oracle(tmp_path):
    """predict(list of HWC BGR ndarrays) and predict(path) = the oracle's preprocess -> predict -> scale_boxes."""
    from PIL import Image
    from oracle import letterbox as olb
    from oracle.postprocess import scale_boxes as oscale
    imgs = _images([(853, 1280), (853, 1280)], 23)
    x = torch.from_numpy(olb.preprocess(imgs))
    ref = oracle().predict(x)
    for r in ref:
        r["boxes"] = r["boxes"].clone()
        oscale(tuple(x.shape[2:]), r["boxes"][:, :4], (853, 1280))
    m = model("n", "f32")
    res = m.predict(imgs)
    assert res[0].orig_shape == (853, 1280) and res[0].orig_img is imgs[0]
    check(ref, res, 0.25, 0.7, 2e-3, 1e-3)  # coordinates scaled by 1/gain = 2
    p = tmp_path / "img.png"
    Image.fromarray(imgs[1][..., ::-1].copy()).save(p)
    rp = m.predict(str(p))
    assert rp[0].path == str(p)
    check(ref[1:], rp, 0.25, 0.7, 2e-3, 1e-3)


def test_batch_independence():
    """An image's detections do not depend on its batch neighbours (per-pixel work only; the tuned tiles may differ
    between B=8 and B=1, so compare with the f32 tolerance)."""
    m = model("n", "f32")
    x = make_input("uniform", tuple(range(71, 79)), 640).to(DEV)
    rb = m.predict(x)
    for i in (0, 5):
        ri = m.predict(x[i:i + 1])
        rep = match_image(rb[i].boxes.data.cpu().numpy(), ri[0].boxes.data.cpu().numpy(), 0.25, 0.7, 1e-3, 1e-3,
                          rep=MatchReport())
        assert rep.ok, rep


def test_segment_plan_f32():
    """yolo11n-seg: Segment head (Proto incl. ConvTranspose2d as a pixel-shuffled GEMM, mask-coefficient branch):
    boxes, classes and the 32 mask coefficients of every kept detection vs the oracle's NMS output."""
    from oracle import postprocess as pp
    x = make_input("uniform", (81,), 640)
    om = oracle("n", "segment")
    _, y, ex = om.raw(x)
    ref = pp.non_max_suppression(y, 0.25, 0.7, nc=80)[0]
    ref[:, :4] = pp.clip_boxes(ref[:, :4].clone(), (640, 640))
    eng = model("n", "f32", "segment").model.engine
    dets, counts = eng.run(x.to(DEV), conf=0.25)
    n = int(counts[0])
    got = dets[0, :n].cpu()
    assert n == len(ref)
    rep = match_image(ref[:, :6].numpy(), got[:, :6].numpy(), 0.25, 0.7, 1e-3, 1e-3, rep=MatchReport())
    assert rep.ok and rep.matched == n, rep
    order_r = torch.argsort(ref[:, 4], descending=True)
    order_g = torch.argsort(got[:, 4], descending=True)
    assert torch.allclose(ref[order_r, 6:], got[order_g, 6:], atol=1e-3, rtol=1e-3)
    proto = eng.read_buffer(eng.graph.proto_buf.id, 1)  # (1, 160, 160, 32) NHWC fp32
    ref_p = ex["proto"].permute(0, 2, 3, 1)
    assert (proto - ref_p).abs().max().item() / ref_p.abs().max().item() < 1e-4


def test_capi_errors():
    from yolomi.lib import Runtime, YMError
    eng = model("n", "f16").model.engine
    args = Runtime.make_args()
    dets, counts = eng.outputs(1, 300)
    x = torch.zeros(1, 3, 100, 100, device=DEV)
    with pytest.raises(YMError, match="EINVAL"):
        eng.rt.infer(x.data_ptr(), 1, 100, 100, args, dets.data_ptr(), counts.data_ptr(), 0)
    with pytest.raises(YMError, match="EINVAL"):
        eng.rt.infer(0, 1, 640, 640, args, dets.data_ptr(), counts.data_ptr(), 0)
    with pytest.raises(YMError, match="EBLOB"):
        Runtime(0, b"\0" * 256)
    with pytest.raises(ValueError):
        model("n", "f16").predict(torch.zeros(1, 3, 100, 96, device=DEV))


def test_results_contract_and_benchmark():
    m = model("n", "f16")
    x = make_input("uniform", (91, 92), 640).to(DEV)
    res = m.predict(x)
    r = res[0]
    assert r.names[0] == "person" and len(r.names) == 80
    assert r.boxes.xyxy.shape[1] == 4 and r.boxes.conf.ndim == 1 and r.boxes.cls.ndim == 1
    for box in r.boxes:  # demo loop (detection_demo.py:116-132)
        cls = int(box.cls[0].item())
        conf = float(box.conf[0].item())
        xyxy = box.xyxy[0].cpu().numpy()
        assert 0 <= cls < 80 and 0.25 < conf <= 1 and xyxy.shape == (4,)
    assert r.orig_img.shape == (640, 640, 3) and r.orig_img.dtype == np.uint8
    b = m.benchmark(x, num_runs=5, warmup_runs=2)
    assert set(b) == {"avg_inference_time", "min_inference_time", "max_inference_time", "fps"}
    info = m.get_model_info()
    assert info["total_parameters"] > 2_000_000 and info["task"] == "detect"


# ------------------------------------------------------------------------------------------------ LDS-DMA conv configs
DMA_FIRST = 17  # csrc/ym_conv.hip: ids >= 17 are the LDS-DMA / split-K kernels of csrc/ym_conv_dma.hip
STREAM_FIRST = DMA_FIRST + 30  # then csrc/ym_conv_stream.hip: 31 streaming 1x1 / 3x3 configs, 12 small-M split-K ones


def _force_cfg(eng, x, cfg):
    """Run once (tables), then pin `cfg` on every conv op for x's shape (inapplicable ops fall back)."""
    eng.run(x, use_graph=False)
    B, _, H, W = x.shape
    eng.rt.set_op_cfg(B, H, W, [cfg if op.kind == "conv" else -1 for op in eng.graph.ops])


HALO_FIRST = STREAM_FIRST + 43  # then csrc/ym_conv_halo.hip: 12 halo-tile 3x3 configs
HALO_CFGS = list(range(HALO_FIRST, HALO_FIRST + 12))


@pytest.mark.parametrize("cfg", list(range(DMA_FIRST, HALO_FIRST)) + HALO_CFGS)
def test_dma_conv_configs_match_oracle(cfg):
    """Every conv of yolo11n (1x1 two-source/upsampled, 3x3 s1/s2, residual, fp32 Detect rows) on one DMA or
    streaming config (ops a config does not apply to fall back to the heuristic choice)."""
    m = model("n", "f16")
    eng = m.model.engine
    x = make_input("uniform", (11, 12), 640)
    _, y, ex = oracle().raw(x, keep=(2, 4, 6, 8, 9, 10, 13, 16, 19, 22))
    xd = x.to(DEV)
    try:
        _force_cfg(eng, xd, cfg)
        eng.run(xd, use_graph=False)
        for b in eng.graph.buffers:
            if b.name.startswith("L") and b.name[1:].isdigit() and int(b.name[1:]) in ex["saved"]:
                ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
                got = eng.read_buffer(b.id, 2)
                rel = (got - ref).abs().max().item() / ref.abs().max().item()
                assert rel < 1e-2, (cfg, b.name, rel)
        no = eng.graph.no
        ref_h = torch.cat([f.view(2, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
        got_h = eng.read_buffer(eng.graph.anchor_buf.id, 2).reshape(2, -1, eng.graph.anchor_buf.C)[..., :no]
        assert (got_h - ref_h).abs().max().item() / ref_h.abs().max().item() < 1e-2
        # graph replay of the same pinned plan is deterministic (split-K reduction order is fixed per tile)
        d1, c1 = eng.run(xd, use_graph=True)
        d1, c1 = d1.clone(), c1.clone()
        d2, c2 = eng.run(xd, use_graph=True)
        assert torch.equal(c1, c2) and torch.equal(d1, d2)
    finally:
        eng._tuned.discard((2, 640, 640))  # the next run reloads the tuned table


def test_dma_split_configs_on_segment_head():
    """yolo11n-seg f16 with a split-K DMA config everywhere: Proto (ConvTranspose2d as a pixel-shuffled GEMM)."""
    x = make_input("uniform", (81,), 640)
    _, y, ex = oracle("n", "segment").raw(x)
    eng = model("n", "f16", "segment").model.engine
    xd = x.to(DEV)
    for cfg in (DMA_FIRST + 4, DMA_FIRST + 29):  # 64x64 split 4, 128x64 split 2
        _force_cfg(eng, xd, cfg)
        eng.run(xd, use_graph=False)
        proto = eng.read_buffer(eng.graph.proto_buf.id, 1)
        ref_p = ex["proto"].permute(0, 2, 3, 1)
        assert (proto - ref_p).abs().max().item() / ref_p.abs().max().item() < 1e-2, cfg


# ------------------------------------------------------------------------------------------------ lanes
@pytest.mark.parametrize("B,lanes", [(8, 2), (8, 4), (3, 2), (1, 4), (5, 3)])
def test_lanes_match_single_lane(B, lanes):
    """Concurrent image slices (parallel graph branches) give the single-lane detections: same NMS input per image,
    the /255 decision still over the whole batch (slices see different kernel batches, hence the f32 tolerance)."""
    eng = model("n", "f32").model.engine
    x = make_input("uniform", tuple(range(101, 101 + B)), 320).to(DEV)
    d1, c1 = eng.run(x, conf=0.1, lanes=1)
    d1, c1 = d1.clone(), c1.clone()
    for use_graph in (True, False):
        d2, c2 = eng.run(x, conf=0.1, lanes=lanes, use_graph=use_graph)
        for i in range(B):
            rep = match_image(d1[i, :int(c1[i])].cpu().numpy(), d2[i, :int(c2[i])].cpu().numpy(), 0.1, 0.7, 1e-3, 1e-3,
                              rep=MatchReport())
            assert rep.ok and rep.matched >= int(c1[i]) - rep.exempt, (i, rep)


def test_lanes_keep_batch_wide_255_rule():
    """One image in [0, 255] makes the whole batch divide by 255 (LoadTensor), even when it sits in another lane."""
    eng = model("n", "f32").model.engine
    x = make_input("uniform", (111, 112, 113, 114), 320).to(DEV)
    x255 = x.clone()
    x255[3] *= 255.0
    d1, c1 = eng.run(x255 / 255.0, conf=0.1, lanes=1)
    d1, c1 = d1.clone(), c1.clone()
    d2, c2 = eng.run(x255, conf=0.1, lanes=2)
    for i in range(4):
        rep = match_image(d1[i, :int(c1[i])].cpu().numpy(), d2[i, :int(c2[i])].cpu().numpy(), 0.1, 0.7, 1e-3, 1e-3,
                          rep=MatchReport())
        assert rep.ok, (i, rep)


# ------------------------------------------------------------------------------------------------ segment masks
def _box_iou(a, b):
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:4], b[None, :, 2:4])
    inter = (rb - lt).clamp(min=0).prod(-1)
    area = lambda t: (t[:, 2] - t[:, 0]) * (t[:, 3] - t[:, 1])
    return inter / (area(a)[:, None] + area(b)[None] - inter)


@pytest.mark.parametrize("scale,seeds", [("n", (81, 82)), ("s", (6001, 6002, 6003, 6004))])
@pytest.mark.parametrize("dtype,agree,min_frac", [("f32", 0.999, 1.0), ("f16", 0.99, 0.9)])
def test_segment_masks_match_oracle(dtype, agree, min_frac, scale, seeds):
    """process_mask(upsample=True) on the GPU vs the oracle (>= 99.9 % pixel agreement on matched
    detections in parity mode); empty masks are dropped on both sides.  yolo11s-seg at B=4 is BASELINE config 5."""
    x = make_input("uniform", seeds, 640)
    ref = oracle(scale, "segment").predict(x, conf=0.25)
    res = model(scale, dtype, "segment").predict(x.to(DEV), conf=0.25)
    total = matched = 0
    for r, g in zip(ref, res):
        rb, gb = r["boxes"], g.boxes.data.cpu()
        assert g.masks is not None and tuple(g.masks.data.shape) == (len(gb), 640, 640)
        assert g.masks.data.dtype == torch.bool and bool(g.masks.data.flatten(1).any(1).all())
        total += len(rb)
        if not len(rb) or not len(gb):
            continue
        iou = _box_iou(rb[:, :4], gb[:, :4])
        iou[rb[:, 5][:, None] != gb[:, 5][None, :]] = 0
        used = set()
        for i in torch.argsort(rb[:, 4], descending=True).tolist():
            j = int(torch.argmax(iou[i]))
            if iou[i, j] < 0.99 or j in used:
                continue
            used.add(j)
            matched += 1
            a = (r["masks"][i] == g.masks.data[j].cpu()).float().mean().item()
            assert a >= agree, (i, j, a)
    assert total > 0 and matched >= min_frac * total - 1, (matched, total)


def test_segment_slot_masks_equal_exact_size_masks():
    """predict()'s single-sync mask path (ym_masks_slots: masks enqueued behind the forward from the device counts)
    and the two-read path it falls back to (ym_masks, exact-size; forced here with a slot cap of 1) give the same
    boxes and the same masks, and the cap grows after a fallback."""
    x = make_input("uniform", (6001, 6002, 6003, 6004), 640).to(DEV)
    m = model("s", "f16", "segment")
    a = m.predict(x, conf=0.25)
    m._mask_cap = 1
    b = m.predict(x, conf=0.25)
    assert m._mask_cap >= max(len(r) for r in b) > 1
    for ra, rb in zip(a, b):
        assert torch.equal(ra.boxes.data, rb.boxes.data)
        assert torch.equal(ra.masks.data, rb.masks.data)
    # over the memory budget the exact-size path runs; the cap follows the counts down again; a mostly
    # empty slot buffer is compacted — all three give the same results
    os.environ["YM_MASK_BUDGET_MB"] = "0"
    try:
        c = m.predict(x, conf=0.25)
    finally:
        del os.environ["YM_MASK_BUDGET_MB"]
    m._mask_cap = 128
    d = m.predict(x, conf=0.25)  # 4 x 128 slots (210 MB), a few dozen kept: compacted
    mx = max(len(r) for r in d)
    assert mx <= m._mask_cap <= 1.25 * mx + 16  # 1.25x the maximum, rounded up to 16
    for ra, rc, rd in zip(a, c, d):
        assert torch.equal(ra.masks.data, rc.masks.data) and torch.equal(ra.masks.data, rd.masks.data)
        assert torch.equal(ra.boxes.data, rc.boxes.data) and torch.equal(ra.boxes.data, rd.boxes.data)


def test_ultralytics_pt_model_path(tmp_path):
    """YOLO11Model(model_path=<Ultralytics .pt>) runs the checkpoint's weights (yolomi/ptimport.py): the same
    detections as a model packed from those (fp16-rounded) weights directly."""
    from core.model import YOLO11Model
    from tests.test_ptimport import _fake_checkpoint
    sd = synth_weights("n", "detect", 3)
    p = tmp_path / "yolo11n.pt"
    _fake_checkpoint(p, sd)
    sd16 = {k: (np.asarray(v).astype(np.float16).astype(np.float32) if np.asarray(v).dtype.kind == "f" else v)
            for k, v in sd.items()}
    x = make_input("uniform", (5,), 640).to(DEV)
    a = YOLO11Model(model_path=str(p), size="n", device="cuda:0", dtype="f32").predict(x)
    b = YOLO11Model(size="n", device="cuda:0", dtype="f32", state_dict=sd16).predict(x)
    assert len(a[0]) == len(b[0]) and torch.equal(a[0].boxes.data, b[0].boxes.data)


# ------------------------------------------------------------------------------------------------ fused conv pairs
SPLIT_TAG = 1 << 20  # csrc/ym_runtime.cpp kSplitTag: op cfg of a fused pair run as its two convs


def test_fused_pairs_split_equals_unfused_plan():
    """The fused f16 plan (yolomi/arch.py fuse_pairs + the C3k cv1 ‖ cv2 merge) with its pairs run as two launches
    (op cfg SPLIT_TAG + ...) and with its pairs on the fused streaming kernel both match the unfused f16 plan on the
    Detect rows within fp16 storage error (the merge and the fused second GEMM change fp32 summation order only)."""
    from core.model import YOLO11Model
    x = make_input("uniform", (5, 6), 640).to(DEV)
    B, _, H, W = x.shape
    os.environ["YM_FUSE"] = "0"
    try:
        mu = YOLO11Model(size="n", device="cuda:0", dtype="f16", verbose=False)
    finally:
        del os.environ["YM_FUSE"]
    eu, ef = mu.model.engine, model("n", "f16").model.engine
    assert not any(op.args.get("pair") for op in eu.graph.ops)
    assert sum(bool(op.args.get("pair")) for op in ef.graph.ops) >= 6
    cfg = 29  # one LDS-DMA config for every conv (inapplicable ops fall back to the heuristic choice)
    eu.run(x, use_graph=False)
    eu.rt.set_op_cfg(B, H, W, [cfg if op.kind == "conv" else -1 for op in eu.graph.ops])
    ef.run(x, use_graph=False)
    fused = ef.rt.get_op_cfg(B, H, W)
    try:
        ef.rt.set_op_cfg(B, H, W, [(SPLIT_TAG + 256 * cfg + cfg if op.args.get("pair") else cfg)
                                   if op.kind == "conv" else -1 for op in ef.graph.ops])
        eu.run(x, use_graph=False)
        ef.run(x, use_graph=False)
        hu = eu.read_buffer(eu.graph.anchor_buf.id, B)
        hs = ef.read_buffer(ef.graph.anchor_buf.id, B)
        ef.rt.set_op_cfg(B, H, W, [(35 if op.args.get("pair") else cfg) if op.kind == "conv" else -1
                                   for op in ef.graph.ops])
        ef.run(x, use_graph=False)
        hf = ef.read_buffer(ef.graph.anchor_buf.id, B)
    finally:
        if fused is not None:
            ef.rt.set_op_cfg(B, H, W, fused)
        ef._tuned.discard((B, H, W))
        eu._tuned.discard((B, H, W))
    rel = lambda a, b: (a - b).abs().max().item() / b.abs().max().item()  # noqa: E731
    assert rel(hs, hu) < 1e-2 and rel(hf, hu) < 1e-2


BNECK_BASE = 17 + 30 + 43 + 12  # csrc/ym_conv.hip: first-gen + DMA + streaming + halo ids, then the Bottleneck kernels
N_BNECK = 14


@pytest.mark.parametrize("scale", ["n", "s"])
def test_bneck_kernel_matches_split_pair(scale):
    """csrc/ym_conv_bneck.hip: every variant (rows x tile width x pixel groups x waves) on every fused Bottleneck of
    the f16 plan — 160x160, 80x80 and (n) 40x40 maps, where 40 is not a multiple of the 16-pixel group — and on every
    stride-2 3x3 -> 1x1 pair (even/odd column layout) equals the same pair run as two conv launches (fp16 mid tensor
    in HBM) within fp16 rounding of the output: the fused kernel rounds the mid tensor to fp16 exactly as the stored
    tensor is, only fp32 summation order differs."""
    m = model(scale, "f16")
    e = m.model.engine
    x = make_input("uniform", (5, 6), 640).to(DEV)
    B, _, H, W = x.shape
    e.run(x, use_graph=False)
    tuned = e.rt.get_op_cfg(B, H, W)
    ops = e.graph.ops
    bn = [i for i, op in enumerate(ops) if op.args.get("pair") and (op.args["pair"]["k"] == 3 or op.args["s"] == 2)]
    assert len(bn) >= 4  # the Bottlenecks and the stride-2 3x3 -> 1x1 pairs (model.1+cv1, n: model.3+cv1)

    def outputs(cfg_bn):
        e.rt.set_op_cfg(B, H, W, [cfg_bn if i in bn else -1 for i in range(len(ops))])
        e.run(x, use_graph=False)
        return [e.read_buffer(ops[i].args["dst"].buf.id, B)[..., ops[i].args["dst"].coff:
                                                               ops[i].args["dst"].coff + ops[i].args["dst"].C]
                for i in bn]

    try:
        ref = outputs(SPLIT_TAG + 256 * 29 + 29)  # the two convs as separate launches (LDS-DMA tiles)
        for v in range(N_BNECK):
            got = outputs(BNECK_BASE + v)
            for i, r, g in zip(bn, ref, got):
                err = (g - r).abs().max().item() / r.abs().max().item()
                assert err < 5e-3, (ops[i].name, v, err)
    finally:
        if tuned is not None:
            e.rt.set_op_cfg(B, H, W, tuned)
        e._tuned.discard((B, H, W))


# ------------------------------------------------------------------------------------------------ BASELINE configs
def _coeff_check(ref_rows, got_rows, conf, iou, tol_xy, tol_s, tol_c, min_frac):
    """NMS rows with mask coefficients: boxes/scores by the matching protocol, then the 32 coefficients of every
    matched pair within tol_c relative to the largest |coefficient|."""
    rep = MatchReport()
    worst = 0.0
    total = 0
    for r, g in zip(ref_rows, got_rows):
        r = np.asarray(r, np.float32).reshape(-1, 38)
        total += len(r)
        before = len(rep.pairs)
        match_image(r[:, :6], g[:, :6], conf, iou, tol_xy, tol_s, rep=rep)
        scale = max(float(np.abs(r[:, 6:]).max()) if len(r) else 1.0, 1e-6)
        for i, j in rep.pairs[before:]:
            worst = max(worst, float(np.abs(r[i, 6:] - g[j, 6:]).max()) / scale)
    if min_frac >= 1.0:
        assert rep.ok, f"{rep}; {rep.failures[:3]}"
    else:
        assert rep.matched + rep.exempt >= min_frac * total, f"{rep}; {rep.failures[:3]}"
    assert worst <= tol_c, (worst, str(rep))
    return rep


@pytest.mark.parametrize("dtype,tol", [("f32", (1e-3, 1e-3, 1e-4, 1e-4, 1.0)), ("f16", (1.0, 1e-2, 2e-2, 1e-2, 0.9))])
def test_segment_s_b4_matches_golden(dtype, tol):
    """BASELINE config 5 — yolo11s-seg, B=4, 640x640 (Proto with 128 channels, the committed f16 tile table
    s-segment-f16-b4): the NMS rows incl. the 32 mask coefficients and the prototypes vs tests/golden/seg_s_uniform."""
    tol_xy, tol_s, tol_c, tol_p, min_frac = tol
    g = json.load(open(os.path.join(GOLD, "seg_s_uniform.json")))
    x = make_input("uniform", g["input"]["seeds"], 640).to(DEV)
    m = model("s", dtype, "segment")
    eng = m.model.engine
    dets, counts = eng.run(x, conf=g["conf"], iou=g["iou"])
    if dtype == "f16":
        assert eng.tune_source[(4, 640, 640)].startswith("committed table")
    got = [dets[b, :int(n)].cpu().numpy() for b, n in enumerate(counts.tolist())]
    _coeff_check(g["nms_rows"], got, g["conf"], g["iou"], tol_xy, tol_s, tol_c, min_frac)
    proto = eng.read_buffer(eng.graph.proto_buf.id, 4).double().reshape(-1)
    p = g["proto"]
    assert abs(float(proto.abs().sum()) - p["abs_sum"]) <= tol_p * p["abs_sum"]
    samples = proto[p["samples_idx"]].numpy()
    assert np.abs(samples - np.array(p["samples"])).max() <= tol_p * max(abs(v) for v in p["samples"])


@pytest.mark.parametrize("scale", ["n", "s"])
def test_committed_b8_f16_tables_match_oracle(scale):
    """BASELINE configs 2 and 3: the f16 plan at B=8 under exactly the committed tile tables the bench runs
    (YM_AUTOTUNE=0: no tuning on the test box), detections and head rows vs the oracle."""
    from core.model import YOLO11Model
    os.environ["YM_AUTOTUNE"] = "0"
    try:
        m = YOLO11Model(size=scale, device="cuda:0", dtype="f16", verbose=False)
    finally:
        del os.environ["YM_AUTOTUNE"]
    x = make_input("uniform", tuple(range(7001, 7009)), 640)
    _, y, ex = oracle(scale).raw(x)
    ref = oracle(scale).predict(x)
    res = m.predict(x.to(DEV))
    eng = m.model.engine
    assert eng.tune_source[(8, 640, 640)] == f"committed table {scale}-detect-f16-b8-640x640.json"
    no = eng.graph.no
    ref_h = torch.cat([f.view(8, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
    got_h = eng.read_buffer(eng.graph.anchor_buf.id, 8).reshape(8, -1, eng.graph.anchor_buf.C)[..., :no]
    assert (got_h - ref_h).abs().max().item() / ref_h.abs().max().item() < 1e-2
    rep = check(ref, res, 0.25, 0.7, 1.0, 1e-2, min_frac=0.9)
    assert rep.matched >= 0.9 * sum(len(r["boxes"]) for r in ref)


def test_sharded_contexts_bitwise_equal_single_context():
    """SURVEY §8(e) on one GPU: two contexts, each on a contiguous 4-image shard of an 8-image batch, with the /255
    decision taken over the GLOBAL batch (yolomi.dist.GlobalBatchMax: each shard's ym_input_max, then MAX — the
    all-reduce of the multi-GPU run), give exactly the single context's detections, image by image (same kernels
    and tile configs: bit-equal).  Image 5, in the second shard only, is 0-255: both shards must divide by 255."""
    from core.model import YOLO11Model
    x = make_input("uniform", tuple(range(7101, 7109)), 640).to(DEV)
    x[5] *= 255.0
    single = model("n", "f16")
    es = single.model.engine
    d1, c1 = es.run(x)
    d1, c1 = d1.clone(), c1.clone()
    cfg8 = es.rt.get_op_cfg(8, 640, 640)
    shards = [YOLO11Model(size="n", device="cuda:0", dtype="f16", weights_blob=es.blob, verbose=False)
              for _ in range(2)]
    maxes = [m.model.engine.input_max(x[4 * r:4 * r + 4]) for r, m in enumerate(shards)]
    gmax = torch.maximum(maxes[0], maxes[1])
    assert float(maxes[0]) <= 1.0 < float(gmax)
    for r, m in enumerate(shards):
        eng = m.model.engine
        if cfg8 is not None:  # the single context's tiles at the shard batch: identical kernels per pixel
            eng.rt.set_op_cfg(4, 640, 640, cfg8)
            eng._tuned.add((4, 640, 640))
        d, c = eng.run(x[4 * r:4 * r + 4], batch_max=gmax)
        for i in range(4):
            n = int(c1[4 * r + i])
            assert int(c[i]) == n, (r, i)
            assert torch.equal(d[i, :n], d1[4 * r + i, :n]), (r, i)
    # without the global statistic, shard 0 alone would NOT divide by 255 (its own max is <= 1)
    d0, c0 = shards[0].model.engine.run(x[:4])
    assert not all(int(c0[i]) == int(c1[i]) and torch.equal(d0[i, :int(c0[i])], d1[i, :int(c1[i])]) for i in range(4))


def _runtime_infer(rt, x, nm=0):
    from yolomi.lib import Runtime
    args = Runtime.make_args(use_graph=True)
    B, _, H, W = x.shape
    dets = torch.zeros((B, 300, 6 + nm), dtype=torch.float32, device=DEV)
    counts = torch.zeros((B,), dtype=torch.int32, device=DEV)
    rt.infer(x.data_ptr(), B, H, W, args, dets.data_ptr(), counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return dets, counts


def test_blob_validation_reload_and_desc():
    """a malformed op record is rejected before anything is committed; a context that already ran can
    load another model (its workspace, graphs and tile tables are dropped); ym_model_desc scale/task/dtype are
    checked against the blob."""
    import struct
    from yolomi.lib import Runtime, YMError
    from yolomi.plan import pack_model
    bn = pack_model("n", "detect", synth_weights("n", "detect", 0), "f16")
    bs = pack_model("s", "detect", synth_weights("s", "detect", 0), "f16")
    for kw in (dict(scale="s"), dict(task="segment"), dict(dtype="f32")):
        with pytest.raises(YMError, match="EBLOB"):
            Runtime(0, bn, **kw)
    h = struct.unpack("<32i", bn[:128])
    nbuf, nop = h[11], h[12]
    for field_, val in ((6, nbuf + 7), (19, 0x7FFFFFF0)):  # src buffer id / weight offset of the first conv record
        bad = bytearray(bn)
        for i in range(nop):
            o = 128 + 32 * nbuf + 128 * i
            if struct.unpack_from("<i", bad, o)[0] == 2:
                struct.pack_into("<i", bad, o + 4 * field_, val)
                break
        with pytest.raises(YMError, match="EBLOB"):
            Runtime(0, bytes(bad))
    x = make_input("uniform", (7201, 7202), 640).to(DEV)
    rt = Runtime(0, bn)
    _runtime_infer(rt, x)
    rt.load(bs)  # reload after a forward: new plan, new buffers
    d, c = _runtime_infer(rt, x)
    d2, c2 = _runtime_infer(Runtime(0, bs), x)
    assert torch.equal(c, c2)
    for b in range(2):
        assert torch.equal(d[b, :int(c[b])], d2[b, :int(c2[b])])


def test_rccl_broadcast_weights_single_rank():
    """ym_broadcast_weights over a one-rank RCCL communicator made by the C-ABI's own bootstrap
    (ym_rccl_get_unique_id / ym_rccl_comm_init): the root path end to end on the device; the context still runs the
    same model afterwards.  (The multi-rank receive path runs in the driver's N-GPU bench.)"""
    from yolomi import lib as L
    from yolomi.plan import pack_model
    bn = pack_model("n", "detect", synth_weights("n", "detect", 0), "f16")
    x = make_input("uniform", (7301,), 640).to(DEV)
    rt = L.Runtime(0, bn)
    d1, c1 = _runtime_infer(rt, x)
    d1, c1 = d1.clone(), c1.clone()
    comm = L.rccl_comm_init(0, 1, L.rccl_unique_id(), 0)
    try:
        rt.broadcast_weights(comm, 0, torch.cuda.current_stream().cuda_stream)
        with pytest.raises(L.YMError, match="EINVAL"):
            rt.broadcast_weights(comm, 1, 0)  # root outside the communicator
    finally:
        L.rccl_comm_destroy(comm)
    d2, c2 = _runtime_infer(rt, x)
    assert torch.equal(c1, c2) and torch.equal(d1[0, :int(c1[0])], d2[0, :int(c2[0])])


@pytest.mark.parametrize("cfg", HALO_CFGS)
def test_halo_conv_configs_yolo11s_b8(cfg):
    """csrc/ym_conv_halo.hip on every applicable 3x3 conv of yolo11s at B=8 (stride 1/2, Cin 16..512, N up to 512,
    residual epilogues, tiles of 1..16 rows): layer outputs and head rows vs the oracle."""
    from core.model import YOLO11Model
    x = make_input("uniform", tuple(range(7401, 7409)), 640)
    _, y, ex = oracle("s").raw(x, keep=(2, 4, 6, 8, 9, 10, 13, 16, 19, 22))
    m = model("s", "f16")
    eng = m.model.engine
    xd = x.to(DEV)
    try:
        _force_cfg(eng, xd, cfg)
        eng.run(xd, use_graph=False)
        for b in eng.graph.buffers:
            if b.name.startswith("L") and b.name[1:].isdigit() and int(b.name[1:]) in ex["saved"]:
                ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
                got = eng.read_buffer(b.id, 8)
                rel = (got - ref).abs().max().item() / ref.abs().max().item()
                assert rel < 1e-2, (cfg, b.name, rel)
        no = eng.graph.no
        ref_h = torch.cat([f.view(8, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
        got_h = eng.read_buffer(eng.graph.anchor_buf.id, 8).reshape(8, -1, eng.graph.anchor_buf.C)[..., :no]
        assert (got_h - ref_h).abs().max().item() / ref_h.abs().max().item() < 1e-2
    finally:
        eng._tuned.discard((8, 640, 640))


def test_decode_staged_variant_bitwise_equals_register_variant():
    """the LDS-staged decode_anchors<false> (any nc / reg_max; forced with YM_DECODE_STAGED=1 in a child
    process, the switch is read once per process) and the register-direct decode_anchors<true> that every
    nc=80 / reg_max=16 plan takes produce the same detections bit for bit."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, torch, numpy as np; sys.path[:0] = [%r, %r];"
            "from tests.golden.make_golden import make_input; from core.model import YOLO11Model;"
            "m = YOLO11Model(size='n', device='cuda:0', dtype='f16');"
            "x = make_input('uniform', (7501, 7502, 7503), 640).cuda();"
            "d, c = m.model.engine.run(x, conf=0.05);"
            "np.save(sys.argv[1], np.concatenate([d[b, :int(c[b])].cpu().numpy() for b in range(3)]))"
            % (os.path.join(root, "yolo-infer_amd"), root))
    outs = []
    for staged in ("0", "1"):
        path = os.path.join(root, "gpurun_out", f"decode_{staged}.npy") if os.path.isdir(
            os.path.join(root, "gpurun_out")) else f"/tmp/decode_{staged}.npy"
        env = dict(os.environ, YM_DECODE_STAGED=staged)
        subprocess.run([sys.executable, "-c", code, path], check=True, env=env, timeout=240)
        outs.append(np.load(path))
    assert outs[0].shape == outs[1].shape and outs[0].shape[0] > 100
    assert np.array_equal(outs[0], outs[1])


# ------------------------------------------------------------------------------------------------ 1280² (N = 1600)
def test_f16_1280_attention_and_layers():
    """benchmark_speed's 1280² size (core/validator.py:188): C2PSA attention over N = 1600 tokens runs the block-wise
    MFMA attention (csrc/ym_misc.hip attn_psa_flash, online softmax) — equal to the scalar kernel within fp16
    rounding, and every checked layer within the f16 plan's 1e-2 of the oracle."""
    import subprocess
    import sys
    x = make_input("uniform", (8001,), 1280)
    _, y, ex = oracle().raw(x, keep=(9, 10, 13, 22))
    m = model("n", "f16")
    eng = m.model.engine
    eng.run(x.to(DEV), use_graph=False)
    l10 = None
    for b in eng.graph.buffers:
        if b.name in ("L9", "L10", "L13", "L22"):
            ref = ex["saved"][int(b.name[1:])].permute(0, 2, 3, 1)
            got = eng.read_buffer(b.id, 1)
            rel = (got - ref).abs().max().item() / ref.abs().max().item()
            assert rel < 1e-2, (b.name, rel)
            if b.name == "L10":
                l10 = got
    # the same layer with the scalar attention kernel (YM_ATTN_FLASH_OFF is read once per process: a child run)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "gpurun_out") if os.path.isdir(os.path.join(root, "gpurun_out")) else "/tmp"
    path = os.path.join(out, "l10_scalar.npy")
    code = ("import sys, numpy as np; sys.path[:0] = [%r, %r];"
            "from tests.golden.make_golden import make_input; from core.model import YOLO11Model;"
            "m = YOLO11Model(size='n', device='cuda:0', dtype='f16'); e = m.model.engine;"
            "e.run(make_input('uniform', (8001,), 1280).cuda(), use_graph=False);"
            "b = [b for b in e.graph.buffers if b.name == 'L10'][0];"
            "np.save(sys.argv[1], e.read_buffer(b.id, 1).numpy())" % (os.path.join(root, "yolo-infer_amd"), root))
    subprocess.run([sys.executable, "-c", code, path], check=True, timeout=240,
                   env=dict(os.environ, YM_ATTN_FLASH_OFF="1"))
    ls = torch.from_numpy(np.load(path))
    assert (ls - l10).abs().max().item() / ls.abs().max().item() < 5e-3


@pytest.mark.parametrize("dtype", ["f32", "f16"])
def test_max_nms_truncation_1280_conf0001(dtype):
    """The validation default conf 0.001 (core/validator.py:91) at 1280²: more than max_nms = 30000 candidates per
    image, so nms_image takes the `n > max_nms` branch (top 30000 by score, csrc/ym_misc.hip) exactly as the oracle's
    argsort[:max_nms] does.  f32 plan: every detection within 1e-3; f16 plan: its own tolerance (1 px / 1e-2)."""
    x = make_input("uniform", (8101,), 1280)
    _, y, _ = oracle().raw(x)
    n_cand = int((y[0, 4:84].amax(0) > 0.001).sum())
    assert n_cand > 30000, n_cand
    ref = oracle().predict(x, conf=0.001)
    res = model("n", dtype).predict(x.to(DEV), conf=0.001)
    if dtype == "f32":
        check(ref, res, 0.001, 0.7, 1e-3, 1e-3)
    else:
        check(ref, res, 0.001, 0.7, 1.0, 1e-2, min_frac=0.9)


NMS_VARIANTS = {"default": {}, "agnostic": {"agnostic": True}, "small_max_wh": {"max_wh": 64.0},
                "classes": {"classes": [0, 2, 5, 9, 14, 27, 41, 56, 63, 79]}}


@pytest.mark.parametrize("variant", list(NMS_VARIANTS))
@pytest.mark.parametrize("dtype,B", [("f32", 2), ("x3", 8)])
def test_nms_blocked_path_equals_per_box_path(dtype, B, variant):
    """csrc/ym_misc.hip nms_image's blocked path (NMS_BM = 512 < candidates <= NMS_BLK_MAX = 12,224 after max_nms:
    keys sorted in LDS, then blocks of NMS_BLK = 256 candidates filtered against the kept list and scanned through
    their own IoU bit matrix) against the one-box-per-barrier path it replaced (ym_set_debug(YM_DBG_NMS, 9)), on the
    same forward's candidates at the validator's conf 0.001 and at 0.02 / 0.004: bit-identical rows and counts (greedy
    NMS is a function of the sorted candidates alone).  Variants: the class filter (cf) applies only when
    boxes of different classes cannot intersect — default max_wh 7680 with and without a `classes` filter (cf on),
    agnostic NMS and max_wh 64 (cf off: every kept box is tested)."""
    from yolomi import lib as L
    kw = NMS_VARIANTS[variant]
    eng = model("n", dtype).model.engine
    x = make_input("uniform", tuple(range(71, 71 + B)), 640).to(DEV)
    for conf in (0.001, 0.004, 0.02):
        d0, c0 = (t.clone() for t in eng.run(x, conf=conf, use_graph=False, **kw))
        if conf == 0.001:  # the blocked path really runs: more than NMS_BM candidates in some image
            logits = eng.read_buffer(eng.graph.anchor_buf.id, B)[:, 0, :, 64:144]
            if "classes" in kw:
                logits = logits[..., kw["classes"]]
            n_cand = int((torch.sigmoid(logits).amax(-1) > conf).sum(-1).max())
            assert n_cand > 512, n_cand
        prev = L.set_debug(L.DBG_NMS, 9)
        try:
            d1, c1 = (t.clone() for t in eng.run(x, conf=conf, use_graph=False, **kw))
        finally:
            L.set_debug(L.DBG_NMS, prev)
        assert torch.equal(c0, c1), (conf, c0.tolist(), c1.tolist())
        for b in range(B):
            n = int(c0[b])
            assert torch.equal(d0[b, :n], d1[b, :n]), (conf, b)
        assert int(c0[:B].max()) > 64  # candidates past the one-wave path
