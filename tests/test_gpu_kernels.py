"""GPU checks of individual kernel variants against a float64 torch reference computed from the kernel's own input
buffer (read back from the plan's arena), so each variant is judged on its own arithmetic, not on upstream error.

Tolerances (written here): fp32-storage plans (f32, x3) within 2e-6 of the output's max magnitude — the kernels
accumulate in fp32 with fmaf, the reference in float64; f16 within 2e-3 (one fp16 rounding of the output)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from bench import synthetic_batch
from yolomi.plan import _dw_weights
from yolomi.synth import synth_weights

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TOL = {"f32": 2e-6, "x3": 2e-6, "f16": 2e-3}


_models = {}


@pytest.mark.parametrize("mode", ["0", "1", "2"])
@pytest.mark.parametrize("scale,B", [("s", 8), ("n", 8), ("s", 1)])
@pytest.mark.parametrize("dtype", ["x3", "f16", "f32"])
def test_dwconv_variants_match_float64(scale, B, dtype, mode):
    """csrc/ym_misc.hip depthwise 3x3 (Detect cv3 DWConv) in each YM_DW_MODE: 0 the LDS-tile kernel
    (default; partial tiles at 20² / 40²), 1 the row variant and one-pixel kernel, 2 the column strips (rows per
    thread 2 or 4 by grid size), on every dwconv of the Detect head at 640² (80², 40², 20² maps), eager forwards:
    output = SiLU(bias + Σ_taps w·x) of the stored input."""
    from core.model import YOLO11Model
    import os
    sd = synth_weights(scale, "detect", 0)
    if (scale, dtype) not in _models:
        os.environ["YM_FUSE_DW"] = "0"  # x3 plans fuse the depthwise ops into their 1x1 convs by default
        try:
            _models[(scale, dtype)] = YOLO11Model(task="detect", size=scale, device="cuda:0", dtype=dtype,
                                                  verbose=False)
        finally:
            del os.environ["YM_FUSE_DW"]
    eng = _models[(scale, dtype)].model.engine
    x = synthetic_batch(B, 640, 77, DEV)
    from yolomi import lib as L
    prev = L.set_debug(L.DBG_DW_MODE, int(mode))
    try:
        eng.run(x, use_graph=False)
    finally:
        L.set_debug(L.DBG_DW_MODE, prev)
    n = 0
    for op in eng.graph.ops:
        if op.kind != "dwconv":
            continue
        a = op.args
        src = eng.read_buffer(a["src"].buf.id, B)[..., a["src"].coff:a["src"].coff + a["C"]]
        got = eng.read_buffer(a["dst"].buf.id, B)[..., a["dst"].coff:a["dst"].coff + a["C"]].double()
        w9, b = _dw_weights(a["wkey"], sd)  # [9][C] fp32, [C]
        C = a["C"]
        w = torch.from_numpy(np.ascontiguousarray(w9.T)).double().reshape(C, 1, 3, 3)
        ref = F.conv2d(src.double().permute(0, 3, 1, 2), w, torch.from_numpy(b).double(), padding=1, groups=C)
        if a["act"]:
            ref = F.silu(ref)
        ref = ref.permute(0, 2, 3, 1)
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < TOL[dtype], (op.name, err)
        n += 1
    assert n == 6


@pytest.mark.parametrize("cfg", [-1, 0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("scale,B,strides", [("s", 8, ""), ("n", 2, ""), ("s", 8, "8,16,32"), ("n", 2, "8,16,32")])
def test_fused_depthwise_1x1_matches_float64(scale, B, strides, cfg):
    """csrc/ym_conv_dwpw.hip (x3 plans: the Detect-head DWConvs fused into the 1x1 conv they feed, yolomi/arch.py
    DW_FUSE_STRIDES; strides "8,16,32" = every level, YM_DW_FUSE_STRIDES) in each configuration (-1: the heuristic;
    0/1/2: tiles 16, 8 or 4 pixels wide; 3-7: the K split over 2-8 workgroups, YM_DWPW_CFGS — a split the op's K
    blocks cannot take falls back to the heuristic), eager forwards: the stored 1x1 output =
    SiLU(b + W · SiLU(b_dw + Σ_taps w_dw·x)) of the stored depthwise input, against float64 with the same fp32
    weights, within 2e-6 of the output's max magnitude (the x3 GEMM's split products miss only lo·lo, ~2^-22)."""
    from core.model import YOLO11Model
    from yolomi.plan import _conv_weights
    import os
    sd = synth_weights(scale, "detect", 0)
    key = (scale, "x3dw", strides)
    if key not in _models:
        if strides:  # (a plan with no committed table: heuristic tiles, no ym_tune here — the test sets the cfgs)
            os.environ["YM_DW_FUSE_STRIDES"] = strides
            os.environ["YM_AUTOTUNE"] = "0"
        try:
            _models[key] = YOLO11Model(task="detect", size=scale, device="cuda:0", dtype="x3", verbose=False)
        finally:
            os.environ.pop("YM_DW_FUSE_STRIDES", None)
            if strides:
                os.environ.pop("YM_AUTOTUNE", None)
    eng = _models[key].model.engine
    x = synthetic_batch(B, 640, 78, DEV)
    eng.run(x, use_graph=False)  # tables for this shape
    try:
        eng.rt.set_op_cfg(B, 640, 640, [cfg if op.args.get("dw") else -1 for op in eng.graph.ops])
        eng.run(x, use_graph=False)
        n = 0
        for op in eng.graph.ops:
            a = op.args
            if not a.get("dw"):
                continue
            C, N = a["c1"], a["c2"]
            src = eng.read_buffer(a["src0"].buf.id, B)[..., a["src0"].coff:a["src0"].coff + C].double()
            got = eng.read_buffer(a["dst"].buf.id, B)[..., a["dst"].coff:a["dst"].coff + N].double()
            w9, bd = _dw_weights(a["dw"]["wkey"], sd)
            wd = torch.from_numpy(np.ascontiguousarray(w9.T)).double().reshape(C, 1, 3, 3)
            h = F.silu(F.conv2d(src.permute(0, 3, 1, 2), wd, torch.from_numpy(bd).double(), padding=1, groups=C))
            w, b = _conv_weights(a, sd)  # (N, 1, 1, C)
            ref = F.conv2d(h, torch.from_numpy(w).double().permute(0, 3, 1, 2), torch.from_numpy(b).double())
            if a["act"]:
                ref = F.silu(ref)
            ref = ref.permute(0, 2, 3, 1)
            err = (got - ref).abs().max().item() / ref.abs().max().item()
            assert err < 2e-6, (op.name, cfg, err)
            n += 1
        assert n == (6 if strides else 2)
    finally:
        eng._tuned.discard((B, 640, 640))


def test_predict_rows_are_per_call():
    """predict() hands the NMS kernel a fresh rows tensor per call (no device copy; a cached graph re-points its NMS
    nodes): Results of earlier calls keep their detections after later calls on other inputs, and the same input
    gives the same rows again (f16 and x3 plans, graph replays, lanes 1 and 2)."""
    from core.model import YOLO11Model
    for dtype, lanes in (("x3", 1), ("f16", 1), ("f16", 2)):
        m = YOLO11Model(task="detect", size="n", device="cuda:0", dtype=dtype, verbose=False)
        m.model.engine.lanes = lanes
        xa, xb = synthetic_batch(4, 320, 5, DEV), synthetic_batch(4, 320, 6, DEV)
        ra = m.predict(xa, conf=0.05)
        da = [r.boxes.data.clone() for r in ra]
        assert sum(len(d) for d in da) > 0
        rb = m.predict(xb, conf=0.05)
        ra2 = m.predict(xa, conf=0.05)
        for r, r2, d in zip(ra, ra2, da):
            assert torch.equal(r.boxes.data, d) and torch.equal(r2.boxes.data, d)
        assert any(not torch.equal(a.boxes.data, b.boxes.data) for a, b in zip(ra, rb))


def test_repointed_graph_rows_with_no_sync_between_calls():
    """a cached forward graph whose NMS nodes are re-pointed (hipGraphExecKernelNodeSetParams) while an
    earlier replay of the same exec may still be in flight.  run(x, dets_out=A) then run(x, dets_out=B) with no
    synchronisation between them: after one sync both hold the same kept rows and neither holds the sentinel."""
    from core.model import YOLO11Model
    m = YOLO11Model(task="detect", size="n", device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    x = synthetic_batch(4, 640, 8, DEV)
    shape = (4, 300, 6)
    warm = torch.empty(shape, dtype=torch.float32, device=DEV)
    eng.run(x, conf=0.05, dets_out=warm)  # capture the graph
    torch.cuda.synchronize()
    for _ in range(3):
        A = torch.full(shape, -7.0, device=DEV)
        B = torch.full(shape, -7.0, device=DEV)
        eng.run(x, conf=0.05, dets_out=A)
        _, counts = eng.run(x, conf=0.05, dets_out=B)
        torch.cuda.synchronize()
        n = counts.tolist()
        assert sum(n) > 0
        for b in range(4):
            assert torch.equal(A[b, :n[b]], B[b, :n[b]]) and torch.equal(A[b, :n[b]], warm[b, :n[b]])
            assert not (A[b, :n[b]] == -7.0).any()


def test_graph_cache_eviction_with_queued_replays():
    """Verdict r4 (a host SIGSEGV inside ym_infer once, with many live contexts): more graph keys than the 16-entry
    cache on one context, every replay still queued when later captures evict earlier graphs (csrc/ym_runtime.cpp
    retire_graph waits for an exec's last launch before destroying it), and three live contexts doing the same in
    turn.  Every call's rows equal the eager forward's bit for bit."""
    from core.model import YOLO11Model
    shape = (1, 300, 6)
    models = [YOLO11Model(task="detect", size="n", device="cuda:0", dtype="x3", verbose=False) for _ in range(3)]
    x = synthetic_batch(1, 640, 12, DEV)
    ref = torch.full(shape, -7.0, device=DEV)
    _, counts = models[0].model.engine.run(x, conf=0.05, use_graph=False, dets_out=ref)
    torch.cuda.synchronize()
    n = int(counts[0])
    assert n > 0
    for m in models:
        eng = m.model.engine
        xs = [x.clone() for _ in range(21)]  # 21 input pointers: 21 graph keys, 5 evictions on this context
        outs = [torch.full(shape, -7.0, device=DEV) for _ in range(2 * len(xs))]
        for i, xi in enumerate(xs + xs[:len(xs)]):  # then the evicted keys again: re-captured behind queued replays
            eng.run(xi, conf=0.05, dets_out=outs[i])
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o[0, :n], ref[0, :n])


def test_async_predict_counts_behind_rows():
    """predict() on a tensor batch does not synchronise: the NMS kernel writes each call's B counts behind its fresh
    rows (ym_infer_args.counts_after_dets) and the Results read them on first access.  Several calls on different
    inputs queued back to back (graph replays, lanes 1 and 2, a side stream current when they are read) give the
    detections of an independent source, bit for bit: the engine's own rows and device counts of an eager forward
    (use_graph=False, no counts-behind-rows), so a wrong counts2 offset cannot hide in the reference."""
    from core.model import YOLO11Model
    for dtype, lanes in (("x3", 1), ("f16", 2)):
        m = YOLO11Model(task="detect", size="n", device="cuda:0", dtype=dtype, verbose=False)
        m.model.engine.lanes = lanes
        xs = [synthetic_batch(3, 320, 40 + i, DEV) for i in range(4)]
        ref = []
        for x in xs:
            d, c = m.model.engine.run(x, conf=0.05, use_graph=False)
            ref.append([d[b, :int(c[b])].clone() for b in range(3)])
        torch.cuda.synchronize()
        got = [m.predict(x, conf=0.05) for x in xs for _ in range(2)]
        with torch.cuda.stream(torch.cuda.Stream()):
            for k, res in enumerate(got):
                assert len(res) == 3
                for r, d in zip(res, ref[k // 2]):
                    assert torch.equal(r.boxes.data, d)
        assert sum(len(d) for d in ref[0]) > 0


def test_predict_on_alternating_streams_is_ordered():
    """every forward of one context shares its arena, NMS scratch, split-K slabs and input_stats ticket,
    so asynchronous predict() calls issued from different torch streams must not overlap.  ym_infer makes a forward
    on another stream than the previous one wait for it (hipStreamWaitEvent on the previous forward's event).  Calls
    alternating between two streams with no synchronisation between them give the same detections as eager
    single-stream forwards of the same inputs."""
    from core.model import YOLO11Model
    m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    xs = [synthetic_batch(4, 640, 60 + i, DEV) for i in range(4)]
    ref = []
    for x in xs:
        d, c = eng.run(x, conf=0.05, use_graph=False)
        ref.append([d[b, :int(c[b])].clone() for b in range(4)])
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = []
    for rep in range(3):
        for k, x in enumerate(xs):
            with torch.cuda.stream(s1 if (k + rep) % 2 == 0 else s2):
                got.append((k, m.predict(x, conf=0.05)))
    for k, res in got:
        for r, d in zip(res, ref[k]):
            assert torch.equal(r.boxes.data, d), k
    assert sum(len(d) for d in ref[0]) > 0


def test_chain_kernel_bitwise_equals_two_launches():
    """DESIGN.md §4.5 (verdict r5 item 1): with YM_DBG_CHAIN = 1 the dependent 20² x3 3x3 pairs that share an LDS-DMA
    configuration (yolo11s B=8: model.8.m.0.m.0.cv1 -> cv2 and their model.22 twins) run as ONE persistent launch
    (csrc/ym_conv_dma.hip conv_dma_chain: per-tile ready counters, write-through hand-off).  The chain launches, and
    every plan buffer and the detections are bit-identical to the two separate launches, eager and graph-replayed."""
    from core.model import YOLO11Model
    from yolomi import lib as L
    m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    x = synthetic_batch(8, 640, 5, DEV)
    d0, c0 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
    nb = len(eng.graph.buffers)
    ref = [eng.read_buffer(b, 8, raw=True) for b in range(nb) if b != eng.graph.input.id]
    prev = L.set_debug(L.DBG_CHAIN, 1)
    L.set_debug(L.DBG_CHAIN_LAUNCHES, 0)
    try:
        d1, c1 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
        got = [eng.read_buffer(b, 8, raw=True) for b in range(nb) if b != eng.graph.input.id]
        n_chain = L.set_debug(L.DBG_CHAIN_LAUNCHES, 0)
        xg = x.clone()  # a new graph key: captured with the chain kernels, replayed three times
        for _ in range(3):
            d2, c2 = (t.clone() for t in eng.run(xg, conf=0.05))
        torch.cuda.synchronize()
    finally:
        L.set_debug(L.DBG_CHAIN, prev)
    assert n_chain >= 1, "no chain kernel launched"
    for r, g in zip(ref, got):
        assert torch.equal(r, g)
    for d, c in ((d1, c1), (d2, c2)):
        assert torch.equal(c0, c)
        for b in range(8):
            assert torch.equal(d0[b, :int(c0[b])], d[b, :int(c0[b])])


def test_stem_fuse_matches_the_split_launches():
    """DESIGN.md §4.5 (verdict r5 item 5): with YM_DBG_STEMFUSE = 1 the x3 stem, model.1 and model.2.cv1 of yolo11s
    run as ONE launch (csrc/ym_stem_fused.hip) that never stores the stem's 320x320 output.  Its stem arithmetic is
    stem_mfma's; model.1 / cv1 sum their K in another order than the split launches, so the pair's output agrees to
    fp32 rounding (max |diff| <= 1e-5 of its max), every later layer to 1e-4, and the detections match the split
    launches' at 5e-4 px / 5e-5 score (the x3 plan's float64 bar), eager and graph-replayed."""
    from core.model import YOLO11Model
    from tests.matching import MatchReport, match_image
    from yolomi import lib as L
    m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    x = synthetic_batch(8, 640, 7, DEV)
    d0, c0 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
    pair = next(op for op in eng.graph.ops if op.name.startswith("model.1+"))
    stem_out = eng.graph.ops[eng.graph.ops.index(pair) - 1].args["dst"].buf.id
    ids = [b for b in range(len(eng.graph.buffers)) if b not in (eng.graph.input.id, stem_out)]
    ref = {b: eng.read_buffer(b, 8) for b in ids}
    prev = L.set_debug(L.DBG_STEMFUSE, 1)
    try:
        d1, c1 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
        got = {b: eng.read_buffer(b, 8) for b in ids}
        xg = x.clone()  # a new graph key: captured with the fused kernel
        for _ in range(2):
            d2, c2 = (t.clone() for t in eng.run(xg, conf=0.05))
        torch.cuda.synchronize()
    finally:
        L.set_debug(L.DBG_STEMFUSE, prev)
    pd = pair.args["dst"].buf.id
    for b in ids:
        scale = float(ref[b].abs().max()) or 1.0
        err = float((got[b] - ref[b]).abs().max()) / scale
        assert err <= (1e-5 if b == pd else 1e-4), (eng.graph.buffers[b].name, err)
    for d, c in ((d1, c1), (d2, c2)):
        rep = MatchReport()
        for b in range(8):
            match_image(d0[b, :int(c0[b])].cpu().numpy(), d[b, :int(c[b])].cpu().numpy(), 0.05, 0.7, 5e-4, 5e-5, rep=rep)
        assert rep.ok and rep.matched > 0, (str(rep), rep.failures[:3])


def test_attention_k_batching_is_bitwise_neutral():
    """YM_DBG_ATTN_KB (csrc/ym_misc.hip attn_psa_x3<NKT, KB>): the x3 C2PSA attention loads the K fragments of every
    key tile at once by default, 8 tiles per round trip with the switch at 1.  Only the load schedule differs, so
    every tensor of the forward and the detections are bitwise equal."""
    from core.model import YOLO11Model
    from yolomi import lib as L
    m = YOLO11Model(task="detect", size="s", device="cuda:0", dtype="x3", verbose=False)
    eng = m.model.engine
    x = synthetic_batch(8, 640, 11, DEV)
    ids = [b for b in range(len(eng.graph.buffers)) if b != eng.graph.input.id]
    prev = L.set_debug(L.DBG_ATTN_KB, 0)
    try:
        d0, c0 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
        ref = {b: eng.read_buffer(b, 8) for b in ids}
        L.set_debug(L.DBG_ATTN_KB, 1)
        d1, c1 = (t.clone() for t in eng.run(x, conf=0.05, use_graph=False))
        got = {b: eng.read_buffer(b, 8) for b in ids}
    finally:
        L.set_debug(L.DBG_ATTN_KB, prev)
    assert any("attn" in op.name for op in eng.graph.ops)
    for b in ids:
        assert torch.equal(ref[b], got[b]), eng.graph.buffers[b].name
    assert torch.equal(c0, c1)
    for b in range(8):
        assert torch.equal(d0[b, :int(c0[b])], d1[b, :int(c1[b])])
