"""CPU tests of the oracle: each restated piece against an independent composition or a hand-computed
expectation.  Parity of the oracle with Ultralytics itself is UNPINNED (no reference tests/fixtures, package not
installable offline) — see oracle/__init__.py and DESIGN.md."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import postprocess as pp
from oracle.yolo11 import DFL, YOLO11, Conv, build, dist2bbox, make_anchors


def test_conv_fuse_matches_unfused():
    torch.manual_seed(0)
    m = Conv(8, 16, 3, 2).eval()
    m.bn.running_mean.uniform_(-0.5, 0.5)
    m.bn.running_var.uniform_(0.5, 2.0)
    m.bn.weight.data.uniform_(0.5, 1.5)
    m.bn.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(2, 8, 32, 32)
    with torch.no_grad():
        ref = F.silu(F.batch_norm(F.conv2d(x, m.conv.weight, None, 2, 1), m.bn.running_mean, m.bn.running_var,
                                  m.bn.weight, m.bn.bias, False, 0.0, 1e-3))
        m.fuse()
        got = m(x)
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-5)


def test_sppf_cascade_identity():
    """max5∘max5 = max9 and max5∘max5∘max5 = max13 with -inf padding (what the fused SPPF kernel relies on)."""
    x = torch.randn(2, 8, 20, 20)
    p5 = lambda t: F.max_pool2d(t, 5, 1, 2)  # noqa: E731
    assert torch.equal(p5(p5(x)), F.max_pool2d(x, 9, 1, 4))
    assert torch.equal(p5(p5(p5(x))), F.max_pool2d(x, 13, 1, 6))


def test_dfl_expectation():
    d = DFL(16)
    logits = torch.zeros(1, 64, 3)
    logits[0, 5, 0] = 50.0  # side 0 of anchor 0: all mass on bin 5
    out = d(logits)
    assert abs(out[0, 0, 0].item() - 5.0) < 1e-4
    assert abs(out[0, 1, 1].item() - 7.5) < 1e-4  # uniform → mean bin 7.5


def test_anchors_and_dist2bbox():
    feats = [torch.zeros(1, 1, 2, 3), torch.zeros(1, 1, 1, 1)]
    pts, st = make_anchors(feats, [8, 16])
    assert pts.tolist() == [[0.5, 0.5], [1.5, 0.5], [2.5, 0.5], [0.5, 1.5], [1.5, 1.5], [2.5, 1.5], [0.5, 0.5]]
    assert st.view(-1).tolist() == [8] * 6 + [16]
    box = dist2bbox(torch.tensor([[1.0, 2.0, 3.0, 4.0]]), torch.tensor([[10.0, 10.0]]), xywh=True)
    assert box.tolist() == [[11.0, 11.0, 4.0, 6.0]]


def _brute_nms(boxes, scores, thr):
    order = sorted(range(len(scores)), key=lambda i: (-scores[i], i))
    keep, sup = [], set()
    for a in order:
        if a in sup:
            continue
        keep.append(a)
        for b in order:
            if b in sup or b == a:
                continue
            x1, y1 = max(boxes[a][0], boxes[b][0]), max(boxes[a][1], boxes[b][1])
            x2, y2 = min(boxes[a][2], boxes[b][2]), min(boxes[a][3], boxes[b][3])
            inter = max(0.0, x2 - x1) * max(0.0, y2 - y1)
            ua = (boxes[a][2] - boxes[a][0]) * (boxes[a][3] - boxes[a][1])
            ub = (boxes[b][2] - boxes[b][0]) * (boxes[b][3] - boxes[b][1])
            if inter / (ua + ub - inter) > thr and order.index(b) > order.index(a):
                sup.add(b)
    return keep


def test_nms_hand_case():
    boxes = torch.tensor([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [0, 0, 10, 10.5]], dtype=torch.float32)
    scores = torch.tensor([0.9, 0.8, 0.7, 0.9])
    keep = pp.nms_greedy(boxes, scores, 0.5).tolist()
    # ties broken by index (stable sort): 0 first, suppresses 3 (IoU 0.952) and 1 (IoU 0.68); 2 survives
    assert keep == [0, 2]


@pytest.mark.parametrize("seed", range(5))
def test_nms_vs_bruteforce(seed):
    g = torch.Generator().manual_seed(seed)
    n = 60
    xy = torch.rand(n, 2, generator=g) * 100
    wh = torch.rand(n, 2, generator=g) * 40 + 1
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(n, generator=g)
    keep = pp.nms_greedy(boxes, scores, 0.5).tolist()
    assert keep == _brute_nms(boxes.tolist(), scores.tolist(), 0.5)


def test_load_tensor_rule():
    x = torch.full((1, 3, 32, 32), 0.5)
    assert torch.equal(pp.load_tensor_check(x), x)
    y = torch.full((1, 3, 32, 32), 2.0)
    assert torch.allclose(pp.load_tensor_check(y), y / 255.0)
    z = torch.full((1, 3, 32, 32), 1.0 + 1.2e-7)  # = 1 + 1 ulp > 1 + eps? eps = 1.19e-7 → 1+eps == 1+ulp
    assert torch.equal(pp.load_tensor_check(z), z)
    with pytest.raises(ValueError):
        pp.load_tensor_check(torch.zeros(1, 3, 33, 32))
    assert pp.load_tensor_check(torch.zeros(3, 32, 32)).shape == (1, 3, 32, 32)


def test_scale_boxes_identity_clip():
    b = torch.tensor([[-5.0, 10.0, 700.0, 641.0]])
    out = pp.scale_boxes((640, 640), b.clone(), (640, 640))
    assert out.tolist() == [[0.0, 10.0, 640.0, 640.0]]


@pytest.mark.parametrize("scale,gflops", [("n", 6.541), ("s", 21.589)])
def test_graph_param_and_flop_counts(scale, gflops):
    import sys
    from yolomi.arch import GraphBuilder
    g = GraphBuilder(scale, "detect")
    assert abs(2 * g.macs_per_image() / 1e9 - gflops) < 1e-3
    m = YOLO11(scale, "detect")
    names = {p.name for p in g.params}
    assert names == set(m.state_dict().keys())
