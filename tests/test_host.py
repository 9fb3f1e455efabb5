"""CPU tests of the host side: synthetic weights, packer, blob, C-ABI exports, facade contract, metrics, matching.
(No compute calls: there is no GPU in this container.)"""
import json
import os
import re
import struct

import numpy as np
import pytest
import torch

from tests.matching import MatchReport, match_image
from yolomi.arch import GraphBuilder, param_specs
from yolomi.metrics import evaluate
from yolomi.plan import MAGIC, fuse_conv_bn, fuse_default, pack_graph, pack_model, x3_weight_exp
from yolomi.synth import splitmix64, synth_weights, uniform

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def test_splitmix64_known_answer():
    # first outputs of splitmix64 from seed 0 (published reference sequence)
    assert [hex(int(v)) for v in splitmix64(0, 3)] == ["0xe220a8397b1dcdaf", "0x6e789e6aa1b965f4",
                                                        "0x6c45d188009454f"]
    u = uniform(7, 1000)
    assert u.min() >= 0 and u.max() < 1 and abs(u.mean() - 0.5) < 0.05


@pytest.mark.parametrize("scale", ["n", "s"])
def test_synth_weights_match_golden(scale):
    g = json.load(open(os.path.join(GOLD, f"weights_{scale}.json")))
    sd = synth_weights(scale, "detect", 0)
    assert set(sd) == set(g["tensors"])
    for k, (s, a) in g["tensors"].items():
        v = sd[k].astype(np.float64)
        assert v.sum() == pytest.approx(s, rel=1e-12, abs=1e-12), k
        assert np.abs(v).sum() == pytest.approx(a, rel=1e-12, abs=1e-12), k


def test_fused_weights_match_oracle_to_one_ulp():
    """The packer's fp32 BN fold (exact elementwise scale·W) equals the oracle's torch fuse_conv_and_bn (diag(scale)
    @ W through the CPU BLAS, which rounds a few channels differently) to ~1e-6 relative."""
    from oracle.yolo11 import build
    sd = synth_weights("n", "detect", 0)
    m = build("n", "detect", sd, fuse=True)
    mods = dict(m.named_modules())
    for p in ("model.0", "model.2.m.0.cv2", "model.10.m.0.attn.pe", "model.23.cv3.1.0.0"):
        w, b = fuse_conv_bn(sd[p + ".conv.weight"], sd[p + ".bn.weight"], sd[p + ".bn.bias"],
                            sd[p + ".bn.running_mean"], sd[p + ".bn.running_var"])
        ref_w, ref_b = mods[p].conv.weight.numpy(), mods[p].conv.bias.numpy()
        np.testing.assert_allclose(w, ref_w, rtol=2e-6, atol=1e-9, err_msg=p)
        np.testing.assert_allclose(b, ref_b, rtol=2e-6, atol=1e-9, err_msg=p)


@pytest.mark.parametrize("scale,task,dtype", [("n", "detect", "f16"), ("s", "segment", "f32")])
def test_blob_layout(scale, task, dtype):
    sd = synth_weights(scale, task, 0)
    blob = pack_model(scale, task, sd, dtype)
    h = struct.unpack("<32i", blob[:128])
    g = GraphBuilder(scale, task, fuse=fuse_default(dtype))
    assert h[0] == MAGIC and h[1] == 1 and h[2] == (0 if dtype == "f16" else 1)
    assert h[3] == (1 if task == "segment" else 0) and h[4] == 80 and h[5] == g.nm and h[6] == 16
    assert h[8:11] == (8, 16, 32) and h[11] == len(g.buffers) and h[12] == len(g.ops)
    meta = 128 + 32 * h[11] + 128 * h[12] + 48 * h[12]
    wb = h[13] | (h[14] << 32)
    assert len(blob) == (meta + 255) // 256 * 256 + wb
    # every conv record: Cin multiple of 8, K padded to the 64-deep kernel step, offsets inside the weight region
    for i in range(h[12]):
        r = struct.unpack("<32i", blob[128 + 32 * h[11] + 128 * i: 128 + 32 * h[11] + 128 * (i + 1)])
        if r[0] == 2:
            assert r[3] % 8 == 0 and r[21] % 64 == 0 and r[21] >= r[1] * r[1] * r[3]
            assert 0 <= r[19] < wb and 0 <= r[20] < wb
            if r[30]:  # fused 1x1 successor: W2 [N2][Kpad2] with K = this conv's N
                assert dtype == "f16" and r[27] > 0 and r[29] % 64 == 0 and r[29] >= r[4]
                assert 0 <= r[25] < wb and 0 <= r[26] < wb


def test_capi_exports_every_declared_symbol():
    import ctypes
    import yolomi.lib as L
    hdr = open(os.path.join(ROOT, "include", "yolomi.h")).read()
    declared = set(re.findall(r"^\s*(?:int|void|const char\*)\s+(ym_\w+)\s*\(", hdr, re.M))
    assert len(declared) >= 15
    lib = ctypes.CDLL(str(L.LIB_PATH))
    for name in declared:
        assert hasattr(lib, name), name
    assert set(L.EXPORTED) == declared
    assert lib.ym_version() == 1
    # int8 (3): conv_i8 + streaming ids, then the LDS-DMA ids in their Q8 mode; fp8 (4): conv_i8 + streaming ids only
    assert lib.ym_num_conv_cfgs(1) == lib.ym_num_conv_cfgs(2) > 100 and 0 < lib.ym_num_conv_cfgs(4) < lib.ym_num_conv_cfgs(3)
    assert lib.ym_num_conv_cfgs(0) < 0
    assert lib.ym_num_conv_cfgs(5) > lib.ym_num_conv_cfgs(1) and lib.ym_num_conv_cfgs(6) < 0  # x3: + its own DMA ids


def test_x3_blob_packs_pair_chunk_weights():
    """x3 plans: every conv but the stem packs [N][Kpad] fp16 rows with each 8-channel K chunk as [hi x8 | lo x8],
    hi = fp16(w), lo = fp16(w - hi) (Kpad = 2K padded to 64); hi + lo restores the fp32 folded weight to ~2^-22
    relative (fp16 subnormal lo parts included); the stem stays fp32.  (Both blobs packed from the graph with C3k
    cv1 ‖ cv2 merged and no fused pairs, so they compare op by op; the x3 pairs' W2: test_x3_fused_pairs_pack_w2.)"""
    sd = synth_weights("n", "detect", 0)
    b32 = pack_graph(GraphBuilder("n", "detect", fuse="merge"), sd, "f32")
    bx3 = pack_graph(GraphBuilder("n", "detect", fuse="merge"), sd, "x3")
    h = struct.unpack("<32i", bx3[:128])
    assert h[2] == 4
    nb, nop = h[11], h[12]
    base = (128 + 32 * nb + 176 * nop + 255) // 256 * 256
    rec = lambda b, i: struct.unpack("<32i", b[128 + 32 * nb + 128 * i: 128 + 32 * nb + 128 * (i + 1)])  # noqa: E731
    worst, nconv = 0.0, 0
    for i in range(nop):
        r32, rx = rec(b32, i), rec(bx3, i)
        if r32[0] != 2:
            continue
        N, Kpad, K = r32[4], r32[21], r32[1] ** 2 * r32[3]
        w = np.frombuffer(b32, np.float32, N * Kpad, base + r32[19]).reshape(N, Kpad)[:, :K]
        if r32[6] == h[15]:  # the stem: fp32 weights, identical
            assert rx[21] == Kpad and np.array_equal(np.frombuffer(bx3, np.float32, N * Kpad, base + rx[19]),
                                                     np.frombuffer(b32, np.float32, N * Kpad, base + r32[19]))
            continue
        assert rx[21] % 64 == 0 and 2 * K <= rx[21] < 2 * K + 64
        hl = np.frombuffer(bx3, np.float16, N * rx[21], base + rx[19]).reshape(N, rx[21])
        assert not hl[:, 2 * K:].any()
        pairs = hl[:, :2 * K].reshape(N, K // 8, 2, 8).astype(np.float64)
        # stored scaled by 2^s, max |w·2^s| in (2^13, 2^14] (so every lo part of a weight above 2^-17 max is normal)
        assert rx[22] == x3_weight_exp(w) and 2 ** 13 < np.abs(w).max() * 2.0 ** rx[22] <= 2 ** 14
        rebuilt = (pairs[:, :, 0] + pairs[:, :, 1]).reshape(N, K) * 2.0 ** -rx[22]
        worst = max(worst, float((np.abs(rebuilt - w) / np.maximum(np.abs(w), 2 ** -17 * np.abs(w).max())).max()))
        nconv += 1
    # every weight to ~2^-22 of ITSELF (unscaled, the subnormal lo parts left ~1e-6 of a typical weight)
    assert nconv > 70 and worst < 2 ** -21


@pytest.mark.parametrize("scale", ["n", "s"])
def test_x3_fused_pairs_pack_w2(scale):
    """x3 plans fuse conv → 1x1 pairs (GraphBuilder fuse="x3": storage K even and within the streaming kernel's K
    steps) and Bottlenecks (3x3 → 3x3 + shortcut); the successor's W2 is packed in pair-chunk rows whose hi + lo
    rebuild the folded fp32 weights to ~2^-22 relative, and Kpad2 counts the fp16 storage K."""
    from yolomi.plan import _conv_weights
    sd = synth_weights(scale, "detect", 0)
    assert fuse_default("x3") == "x3"
    g = GraphBuilder(scale, "detect", fuse="x3")
    pairs = [op for op in g.ops if op.args.get("pair")]
    assert pairs and any(op.args["pair"]["k"] == 3 for op in pairs) and any(op.args["pair"]["k"] == 1 for op in pairs)
    assert any(op.name == "model.1+cv1" for op in pairs)
    blob = pack_model(scale, "detect", sd, "x3")
    h = struct.unpack("<32i", blob[:128])
    nb, nop = h[11], h[12]
    assert nop == len(g.ops)
    base = (128 + 32 * nb + 176 * nop + 255) // 256 * 256
    for i, op in enumerate(g.ops):
        r = struct.unpack("<32i", blob[128 + 32 * nb + 128 * i: 128 + 32 * nb + 128 * (i + 1)])
        assert bool(r[30]) == bool(op.args.get("pair")), op.name
        if not r[30]:
            continue
        w2, _ = _conv_weights(op.args["pair"], sd)
        N2, K2 = w2.shape[0], w2.shape[1] * w2.shape[2] * w2.shape[3]
        assert r[27] == N2 and r[29] % 64 == 0 and 2 * K2 <= r[29] < 2 * K2 + 64 and (r[29] // 32) % 2 == 0
        hl = np.frombuffer(blob, np.float16, N2 * r[29], base + r[25]).reshape(N2, r[29])
        pr = hl[:, :2 * K2].reshape(N2, K2 // 8, 2, 8).astype(np.float64)
        ref = w2.reshape(N2, K2)
        assert r[23] == x3_weight_exp(ref), op.name
        rebuilt = (pr[:, :, 0] + pr[:, :, 1]).reshape(N2, K2) * 2.0 ** -r[23]
        rel = np.abs(rebuilt - ref) / np.maximum(np.abs(ref), 2 ** -17 * np.abs(ref).max())
        assert rel.max() < 2 ** -21, op.name

@pytest.mark.parametrize("scale", ["n", "s"])
def test_x3_fused_depthwise_pack(scale, monkeypatch):
    """x3 plans merge the Detect-head DWConvs of the P3 maps into the 1x1 conv that consumes them (GraphBuilder.fuse_dw;
    P4 / P5 measured slower fused): the fused conv reads the depthwise INPUT, keeps the 1x1's weights and carries the depthwise
    [9][C] weights ‖ bias at record slot 24 (1 + offset); YM_FUSE_DW=0 keeps the six depthwise launches."""
    from yolomi.plan import _dw_weights
    sd = synth_weights(scale, "detect", 0)
    g0 = GraphBuilder(scale, "detect", fuse=False)
    g = GraphBuilder(scale, "detect", fuse="x3")
    assert len([op for op in g.ops if op.kind == "dwconv"]) == 4  # the P4 / P5 ones (GraphBuilder.DW_FUSE_STRIDES)
    fused = [op for op in g.ops if op.args.get("dw")]
    assert len(fused) == 2 and len([op for op in g0.ops if op.kind == "dwconv"]) == 6
    assert all(op.args["src0"].buf.f == 8 for op in fused)
    assert g.macs_per_image() == g0.macs_per_image()
    dws = {op.name: op for op in g0.ops if op.kind == "dwconv"}
    for op in fused:
        d = dws[op.name.split("+")[0]]
        assert op.args["src0"].buf.name == d.args["src"].buf.name and op.args["c1"] == d.args["C"]
        assert op.args["k"] == 1 and not op.args.get("pair")
    blob = pack_model(scale, "detect", sd, "x3")
    h = struct.unpack("<32i", blob[:128])
    nb, nop = h[11], h[12]
    base = (128 + 32 * nb + 176 * nop + 255) // 256 * 256
    for i, op in enumerate(g.ops):
        r = struct.unpack("<32i", blob[128 + 32 * nb + 128 * i: 128 + 32 * nb + 128 * (i + 1)])
        assert (r[24] > 0) == bool(op.args.get("dw")), op.name
        if r[24] > 0:
            C = op.args["c1"]
            w9, b = _dw_weights(op.args["dw"]["wkey"], sd)
            got = np.frombuffer(blob, np.float32, 10 * C, base + r[24] - 1)
            assert np.array_equal(got[:9 * C], w9.reshape(-1)) and np.array_equal(got[9 * C:], b.astype(np.float32))
    monkeypatch.setenv("YM_FUSE_DW", "0")
    assert len([op for op in GraphBuilder(scale, "detect", fuse="x3").ops if op.kind == "dwconv"]) == 6


def test_facade_contract_without_gpu():
    from core.model import YOLO11Model
    with pytest.raises(ValueError):
        YOLO11Model(task="bogus", device="cuda")
    with pytest.raises(ValueError):
        YOLO11Model(size="q", device="cuda")
    with pytest.raises(NotImplementedError):
        YOLO11Model(task="classify", device="cuda")
    with pytest.raises(RuntimeError, match="no HIP path"):
        YOLO11Model(device="cpu")  # no silent CPU fallback
    assert set(YOLO11Model.SUPPORTED_TASKS) == {"detect", "segment", "classify", "pose", "obb"}


def test_param_count_matches_ultralytics_cards():
    # fused parameter counts (conv weights + biases) — SURVEY §0 table
    for scale, expect in (("n", 2_616_232), ("s", 9_443_744)):
        sd = synth_weights(scale, "detect", 0)
        n = 0
        for k, v in sd.items():
            if k.endswith(".conv.weight") and "dfl" not in k:  # conv + its folded BN bias
                n += v.size + v.shape[0]
            elif k.endswith(".weight") and ".bn." not in k and ".conv." not in k:  # plain Conv2d heads
                n += v.size
            elif k.endswith(".bias") and ".bn." not in k:
                n += v.size
        assert n == expect


def test_metrics_map():
    gt = [np.array([[10, 10, 50, 50, 1, 3], [100, 100, 150, 180, 1, 5]], np.float64)]
    # perfect predictions score 0.995 under the 101-point interpolation + trapezoid rule (the Ultralytics value)
    assert evaluate([gt[0].copy()], gt)["map"] == pytest.approx(0.995)
    shifted = gt[0].copy()
    shifted[1, :4] += 20  # IoU of the second box drops to ~0.4: below every threshold
    m = evaluate([shifted], gt)
    assert 0.4 < m["map"] < 0.6 and m["map50"] == pytest.approx(0.4975)
    assert evaluate([np.zeros((0, 6))], gt)["map"] == 0.0


def test_match_predictions_prediction_order_known_answer():
    """One ground truth, two same-class candidates: upstream match_predictions keeps, per ground truth, the first
    remaining pair in PREDICTION order (the more confident prediction, IoU 0.6), not the higher-IoU one (0.9) — the
    IoU re-sort between its two unique() steps is commented out upstream.  At t >= 0.65 only the IoU-0.9 prediction
    qualifies."""
    from yolomi.metrics import IOUV, match_predictions
    gt = np.array([[0, 0, 100, 100, 1, 7]], np.float64)
    p0 = [0, 0, 100, 60, 0.9, 7]   # IoU 0.6
    p1 = [0, 0, 100, 90, 0.8, 7]   # IoU 0.9
    tp = match_predictions(np.array([p0, p1], np.float64), gt)
    k50, k65 = 0, int(np.argmin(np.abs(IOUV - 0.65)))
    assert tp[0, k50] and not tp[1, k50]
    assert not tp[0, k65] and tp[1, k65]
    assert tp[1, int(np.argmin(np.abs(IOUV - 0.9)))] and not tp[:, -1].any()


def test_matching_protocol():
    ref = np.array([[0, 0, 10, 10, 0.9, 1], [20, 20, 40, 40, 0.2505, 2]], np.float32)
    got = np.array([[0, 0, 10, 10.0005, 0.9002, 1]], np.float32)
    rep = match_image(ref, got, 0.25, 0.7, 1e-3, 1e-3, rep=MatchReport())
    assert rep.matched == 1 and rep.exempt == 1 and rep.ok  # 0.2505 is within 2e-3 of conf
    bad = np.array([[0, 0, 10, 10, 0.9, 2]], np.float32)  # wrong class
    assert not match_image(ref[:1], bad, 0.25, 0.7, 1e-3, 1e-3, rep=MatchReport()).ok


def test_validator_benchmark_schema(tmp_path):
    from core.validator import YOLO11Validator

    class FakeModel:
        def get_model_info(self):
            return {"task": "detect", "size": "n"}

        def benchmark(self, data_source, num_runs=100, warmup_runs=10):
            return {"avg_inference_time": 0.002, "min_inference_time": 0.001, "max_inference_time": 0.003,
                    "fps": 500.0}

    v = YOLO11Validator(FakeModel(), device="cpu", output_dir=tmp_path)
    r = v.benchmark_speed(None, num_runs=2, warmup_runs=1, batch_sizes=[1, 8], image_sizes=[320, 640])
    assert set(r) == {"device", "model_info", "configurations", "summary"}
    assert len(r["configurations"]) == 4
    c = r["configurations"][1]
    assert set(c) == {"avg_inference_time", "min_inference_time", "max_inference_time", "fps", "batch_size",
                      "image_size", "images_per_second"}
    assert c["images_per_second"] == 8 * 500.0
    assert set(r["summary"]) == {"best_fps", "avg_fps", "best_latency", "avg_latency", "best_throughput",
                                 "total_configurations_tested", "best_configuration"}
    assert (tmp_path / "benchmark_results.json").exists() and (tmp_path / "benchmark_summary.txt").exists()


def test_op_costs_cover_all_flops():
    g = GraphBuilder("n", "detect")
    costs = g.op_costs(8, 640, 640)
    conv_flops = sum(c[0] for c, op in zip(costs, g.ops) if op.kind in ("conv", "dwconv", "attn"))
    assert conv_flops == pytest.approx(8 * 2 * g.macs_per_image(640, 640), rel=1e-9)
    assert len(param_specs("n")) == 499


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_dma_kernels_issue_exactly_the_counted_loads():
    """The LDS-DMA conv kernels' counted vmcnt waits assume 3·(BM/32 + BN/32) DMA instructions per kernel."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_dma_asm.py")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_save_detection_results_formats(tmp_path):
    """utils.visualization.save_detection_results writes the reference's txt/json/csv formats
    (/root/reference/utils/visualization.py:342-437): checked against a per-box restatement of those formats."""
    import csv as _csv
    from core.results import Results
    from utils.visualization import save_detection_results
    rng = np.random.default_rng(9)
    d = torch.from_numpy(np.concatenate([rng.uniform(0, 640, (5, 4)), rng.uniform(0.25, 1, (5, 1)),
                                         rng.integers(0, 80, (5, 1))], 1).astype(np.float32))
    r = Results(torch.zeros(3, 64, 64), {i: str(i) for i in range(80)}, d)
    per_box = [(int(b.cls[0].item()), float(b.conf[0].item()), [float(v) for v in b.xyxy[0].tolist()]) for b in r.boxes]
    save_detection_results(r, str(tmp_path / "o" / "a.txt"), "txt")
    want = "".join(f"{c} {s:.6f} {x[0]:.6f} {x[1]:.6f} {x[2]:.6f} {x[3]:.6f}\n" for c, s, x in per_box)
    assert (tmp_path / "o" / "a.txt").read_text() == want
    save_detection_results(r, str(tmp_path / "a.json"), "json")
    got = json.loads((tmp_path / "a.json").read_text())
    assert got == {"detections": [{"class_id": c, "confidence": s, "bbox": x} for c, s, x in per_box]}
    save_detection_results(r, str(tmp_path / "a.csv"), "CSV")
    rows = list(_csv.reader(open(tmp_path / "a.csv")))
    assert rows[0] == ["class_id", "confidence", "x1", "y1", "x2", "y2"]
    assert rows[1:] == [[str(c), str(s)] + [str(v) for v in x] for c, s, x in per_box]
    empty = Results(torch.zeros(3, 64, 64), {}, torch.zeros(0, 6))
    save_detection_results(empty, str(tmp_path / "e.csv"), "csv")
    assert len(list(_csv.reader(open(tmp_path / "e.csv")))) == 1
    with pytest.raises(ValueError):
        save_detection_results(r, str(tmp_path / "a.xml"), "xml")


@pytest.mark.parametrize("scale,task", [("n", "detect"), ("s", "detect"), ("s", "segment")])
def test_fused_pairs(scale, task):
    """GraphBuilder.fuse_pairs: each fused op is a conv followed by a 1x1 conv (or, for a Bottleneck, a 3x3 conv)
    that was the only reader of the conv's output; the work (MACs) is unchanged, the intermediate tensor leaves the byte count and no op reads it."""
    g0, g = GraphBuilder(scale, task), GraphBuilder(scale, task, fuse=True)
    pairs = [op for op in g.ops if op.args.get("pair")]
    names0 = [op.name for op in g0.ops]
    merged = [op for op in g.ops if op.args.get("wkeys")]  # C3k cv1 ‖ cv2
    assert [op.name for op in merged] == [f"model.{i}.m.0.cv1+cv2" for i in (6, 8, 22)]
    assert len(g.ops) == len(g0.ops) - len(pairs) - len(merged)
    assert g.macs_per_image() == g0.macs_per_image()
    heads = {f"model.23.cv2.{l}.1+2" for l in range(3)} | {f"model.23.cv3.{l}.1.1+2" for l in range(3)}
    assert heads <= {op.name for op in pairs}
    for op in pairs:
        first = op.name.split("+")[0]
        i = names0.index(first)
        nxt = g0.ops[i + 1]
        assert nxt.args["k"] == op.args["pair"]["k"] and nxt.args["src0"].buf.name == op.args["pair"]["mid"].buf.name
        if op.args["pair"]["k"] == 3:  # a Bottleneck: both 3x3, the shortcut is the first conv's input
            assert op.args["k"] == 3 and op.args["res"] is not None
            assert (op.args["res"].buf.name, op.args["res"].coff) == (op.args["src0"].buf.name, op.args["src0"].coff)
        assert (op.args["dst"].buf.name, op.args["dst"].coff) == (nxt.args["dst"].buf.name, nxt.args["dst"].coff)
        mid = op.args["pair"]["mid"].buf
        for o in g.ops:
            for k in ("src0", "src1", "res", "src", "qkv"):
                v = o.args.get(k)
                assert not (v is not None and hasattr(v, "buf") and v.buf is mid), (op.name, o.name)
    c0, c1 = g0.op_costs(8, 640, 640), g.op_costs(8, 640, 640)
    assert sum(c[0] for c in c0) == sum(c[0] for c in c1)
    saved = sum(c[1] for c in c0) - sum(c[1] for c in c1)
    mids = sum(op.args["pair"]["mid"].C * 8 * (640 // g.out_factor(op)) ** 2 * 2 * 2 for op in pairs)
    xs = sum(op.args["src0"].C * 8 * (640 // g.out_factor(op)) ** 2 * 2 for op in merged)
    assert saved == mids + xs  # each intermediate was written and read once, each merged input read once, at 2 B
    with pytest.raises(ValueError):
        GraphBuilder(scale, task, quant=True, fuse=True)


def test_checkpoint_architecture_is_inferred_and_mismatches_rejected():
    """a checkpoint decides the plan (reference YOLO(model_path), core/model.py:100-110); packing a
    state dict into a graph of another scale or class count fails loudly instead of writing past buffers."""
    from yolomi.arch import infer_arch
    from yolomi.plan import pack_graph
    sd_s = synth_weights("s", "detect", 0)
    assert infer_arch(sd_s) == ("s", "detect", 80)
    assert infer_arch(synth_weights("n", "segment", 0)) == ("n", "segment", 80)
    with pytest.raises(ValueError, match="shape"):
        pack_graph(GraphBuilder("n", "detect"), sd_s, "f16")
    # a 20-class checkpoint: the cls branch width c3 = max(ch0, min(nc, 100)) changes with nc too
    rng = np.random.default_rng(0)
    g20 = GraphBuilder("n", "detect", nc=20)
    sd20 = {p.name: (rng.standard_normal(p.shape).astype(np.float32) * 0.1 if p.kind not in ("bn_var", "count")
                     else np.ones(p.shape, np.float32)) for p in g20.params}
    assert infer_arch(sd20) == ("n", "detect", 20)
    pack_graph(g20, sd20, "f16")
    with pytest.raises(ValueError, match="shape"):
        pack_graph(GraphBuilder("n", "detect"), sd20, "f16")
    blob = pack_model("s", "detect", sd_s, "f16")
    assert struct.unpack("<32i", blob[:128])[19] == ord("s")  # ym_model_desc.scale is checked against this


def test_resource_monitor_contract():
    """utils/helpers.ResourceMonitor keeps the reference's data-point keys and averages (helpers.py:715-834); on a
    host without a GPU driver the AMD SMI side degrades to an empty gpu_usage list."""
    import time as _t
    from utils.helpers import ResourceMonitor
    m = ResourceMonitor(interval=0.05)
    m.start_monitoring()
    _t.sleep(0.5)
    m.stop_monitoring()
    assert len(m.history) >= 2
    p = m.get_current_usage()
    assert {"timestamp", "cpu_percent", "memory_percent", "memory_used", "memory_total", "gpu_usage"} <= set(p)
    avg = m.get_average_usage()
    assert "avg_cpu_percent" in avg and "avg_memory_percent" in avg


def test_x3_weight_exp_is_clamped_to_the_loader_range():
    """a nearly pruned conv (max |w| < 2^-50) must still pack into a blob ym_load_weights accepts
    (|s| <= 64, csrc/ym_runtime.cpp conv_args), and a huge one too; ordinary matrices keep max |w·2^s| in (2^13, 2^14]."""
    from yolomi.plan import X3_WEXP_MAX
    assert x3_weight_exp(np.full((8, 8), 2.0 ** -60, np.float32)) == X3_WEXP_MAX
    assert x3_weight_exp(np.full((8, 8), 2.0 ** 90, np.float32)) == -X3_WEXP_MAX
    w = np.full((8, 8), 0.03, np.float32)
    assert 2 ** 13 < 0.03 * 2.0 ** x3_weight_exp(w) <= 2 ** 14
    assert x3_weight_exp(np.zeros((8, 8), np.float32)) == 0
