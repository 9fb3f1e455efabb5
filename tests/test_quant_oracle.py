"""CPU tests of the int8 PTQ restatement (oracle/quant.py) and of the product's int8 packing (yolomi.quant/plan).

Pins: the restated quantized conv against torch.ao's own quantized::conv2d kernels (the kernels the reference's
PostTrainingQuantizer converts to, /root/reference/optimization/quantization/quantizers.py:77) on real layers of the
synthetic model; the float walk against the oracle's forward; the quantisation-point names shared by the oracle and
the GPU plan; the product's weight fold/quantisation against the oracle's (bit-exact); the committed int8 fixtures.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import quant as Q
from oracle.predict import OracleModel
from tests.golden.make_golden import I8_FIXTURES, LAYERS, make_input
from tests.matching import MatchReport, match_image
from yolomi.arch import GraphBuilder
from yolomi.synth import synth_weights

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_cache = {}


def sd_n(task="detect"):
    if task not in _cache:
        _cache[task] = synth_weights("n", task, 0)
    return _cache[task]


def test_float_walk_is_the_oracle_forward():
    sd = sd_n()
    x = make_input("uniform", (7,), 320)
    om = OracleModel("n", "detect", sd)
    _, y0, _ = om.raw(x)
    y1, _, _ = Q.float_walk(om.net, x)
    assert torch.equal(y0, y1)


def test_elementwise_fold_matches_oracle_fuse():
    """The int8 path folds BN elementwise; the float oracle folds with Ultralytics' diag-matrix product: equal to
    ~1 ulp (the detections of the float path are unaffected)."""
    sd = sd_n()
    a = dict(Q.build_folded("n", "detect", sd).named_modules())
    b = dict(OracleModel("n", "detect", sd).net.named_modules())
    for p in ("model.0", "model.2.m.0.cv2", "model.10.m.0.attn.pe", "model.23.cv3.1.0.0"):
        torch.testing.assert_close(a[p].conv.weight, b[p].conv.weight, rtol=2e-6, atol=1e-9)
        torch.testing.assert_close(a[p].conv.bias, b[p].conv.bias, rtol=2e-6, atol=1e-9)


def test_product_fold_and_weight_quantisation_are_bit_exact():
    """yolomi.plan (numpy fold) + yolomi.quant.quantize_weight produce exactly the oracle's int8 weights."""
    from yolomi.plan import _conv_weights, _dw_weights
    from yolomi.quant import quantize_weight as pq
    sd = sd_n()
    mods = dict(Q.build_folded("n", "detect", sd).named_modules())
    g = GraphBuilder("n", "detect", quant=True)
    ops = {op.name: op for op in g.ops}
    for p in ("model.0", "model.2.m.0.cv2", "model.9.cv2", "model.23.cv2.0.2"):
        w, b = _conv_weights(ops[p].args, sd)  # (N, k, k, cin)
        conv = mods[p].conv if hasattr(mods[p], "conv") else mods[p]
        assert np.array_equal(np.transpose(w, (0, 3, 1, 2)), conv.weight.numpy()), p
        assert np.array_equal(b, conv.bias.numpy()), p
        for pc in (False, True):
            q1, s1 = pq(w, pc)
            q2, s2 = Q.quantize_weight(conv.weight, pc)
            assert np.array_equal(np.transpose(q1, (0, 3, 1, 2)), q2.numpy().astype(np.int8)), (p, pc)
            assert np.array_equal(s1, s2), (p, pc)
    w9, _ = _dw_weights("model.23.cv3.0.0.0", sd)
    assert np.array_equal(w9.T.reshape(-1, 1, 3, 3), mods["model.23.cv3.0.0.0"].conv.weight.numpy())


@pytest.mark.parametrize("task", ["detect", "segment"])
def test_quantisation_points_shared_with_the_plan(task):
    sd = sd_n(task)
    net = Q.build_folded("n", task, sd)
    qp = Q.calibrate(net, [make_input("uniform", (3,), 64)], "qnnpack")
    okeys = set(qp) - {"backend"}
    for quant in (False, True):
        g = GraphBuilder("n", task, quant=quant)
        keys = {b.qkey for b in g.buffers if b.qname}
        keys |= {"out:" + op.args["wkey"] for op in g.ops if op.kind in ("conv", "dwconv", "attn")}
        keys |= {"act:" + op.args["catq"] for op in g.ops if op.kind == "conv" and op.args.get("catq")}
        assert keys == okeys, (quant, sorted(keys ^ okeys)[:8])


@pytest.mark.parametrize("backend,layer", [("qnnpack", "model.1"), ("qnnpack", "model.2.m.0.cv2"),
                                           ("fbgemm", "model.3"), ("qnnpack", "model.23.cv3.0.0.0")])
def test_quantized_conv_matches_torch_ao_kernel(backend, layer):
    """The restated quantized conv vs torch.ops.quantized.conv2d (the engine the reference's qconfig selects) on a real
    layer: identical int8 outputs except rare round-half ties (the engines requantise in their own fp32 order)."""
    if backend not in torch.backends.quantized.supported_engines:
        pytest.skip(f"{backend} engine not built into this torch")
    sd = sd_n()
    net = Q.build_folded("n", "detect", sd)
    mods = dict(net.named_modules())
    conv = mods[layer].conv
    ctx = Q._Ctx(backend, "quant", {})
    torch.manual_seed(0)
    cin = conv.in_channels
    xq = torch.randint(ctx.qmin, ctx.qmax + 1, (1, cin, 24, 24)).float()
    s_in, z_in = 0.02, int(ctx.qmax // 5)
    with torch.no_grad():
        y = torch.nn.functional.conv2d((xq - z_in) * s_in, conv.weight, conv.bias, conv.stride, conv.padding,
                                       conv.dilation, conv.groups)
    s_out = float(np.float32((y.max() - y.min()).item() / ctx.qmax))
    z_out = int(round(float(-y.min() / s_out)))
    ctx.qp["out:" + layer] = (s_out, z_out)
    _, st = ctx.conv(layer, conv, Q.QT(xq, s_in, z_in), False)
    prev = torch.backends.quantized.engine
    torch.backends.quantized.engine = backend
    try:
        wq, sw = ctx.weights(layer, conv)
        qx = torch._make_per_tensor_quantized_tensor(xq.to(torch.uint8), Q.F32(s_in).item(), z_in)
        if ctx.per_channel:
            qw = torch._make_per_channel_quantized_tensor(wq.to(torch.int8), torch.from_numpy(sw).double(),
                                                          torch.zeros(len(sw), dtype=torch.long), 0)
        else:
            qw = torch._make_per_tensor_quantized_tensor(wq.to(torch.int8), float(sw[0]), 0)
        packed = torch.ops.quantized.conv2d_prepack(qw, conv.bias.detach().float(), list(conv.stride),
                                                    list(conv.padding), list(conv.dilation), conv.groups)
        ref = torch.ops.quantized.conv2d(qx, packed, s_out, z_out).int_repr().float()
    finally:
        torch.backends.quantized.engine = prev
    d = (ref - st.q).abs()
    assert d.max() <= 1 and float((d > 0).float().mean()) < 5e-3, (float(d.max()), float((d > 0).float().mean()))


@pytest.mark.parametrize("backend", ["qnnpack", "fbgemm"])
def test_int8_blob_packs(backend):
    from yolomi.plan import pack_model
    sd = sd_n()
    qp = Q.calibrate(Q.build_folded("n", "detect", sd), [make_input("uniform", (4,), 64)], backend)
    blob = pack_model("n", "detect", sd, "i8", qp)
    assert int.from_bytes(blob[8:12], "little") == 2  # dtype i8
    with pytest.raises(ValueError):
        pack_model("n", "detect", sd, "i8", None)


@pytest.mark.parametrize("name", list(I8_FIXTURES))
def test_int8_oracle_reproduces_golden(name):
    g = json.load(open(os.path.join(GOLD, name + ".json")))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    qp = Q.qparams_from_json(g["qparams"])
    m = Q.Int8OracleModel(g["scale"], "detect", synth_weights(g["scale"], "detect", g["weights_seed"]), qp)
    x = make_input(g["input"]["kind"], g["input"]["seeds"], g["input"]["size"])
    im, y, ex = m.raw(x)
    for i in LAYERS:
        t = ex["stored"][i].q.permute(0, 2, 3, 1).double()
        ref = g["layers"][f"L{i}"]
        assert float(t.sum()) == ref["sum"], i  # integers: exact
    dets = m.predict(x, conf=g["conf"], iou=g["iou"])
    rep = MatchReport()
    for d, r in zip(dets, g["dets"]):
        match_image(np.array(r, np.float32).reshape(-1, 6), d["boxes"].numpy(), g["conf"], g["iou"], 1e-3, 1e-4,
                    rep=rep)
    assert rep.ok, rep.failures[:3]
