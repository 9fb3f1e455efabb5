"""Image-source preprocessing: the letterbox oracle and the host geometry on the CPU.

The oracle (oracle/letterbox.py) restates Ultralytics LetterBox + OpenCV's scalar fixed-point INTER_LINEAR; parity with
cv2 itself is unpinned (no OpenCV here).  It is pinned by the Ultralytics geometry known answer of SURVEY §8f
(image.jpg 1280x853 -> a 640x448 canvas), by exact identities (identity size, constant images) and by agreement with
torch's bilinear resize (align_corners=False, the same sampling grid) to within one level.  The GPU kernel is
checked against the oracle bit for bit in tests/test_gpu_parity.py.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import letterbox as olb
from yolomi import preprocess as pp


def test_geometry_known_answer():
    # /root/reference/image.jpg (1280 x 853) letterboxes to 640 x 448 with auto=True, stride 32
    uh, uw, t, b, l, r = olb.letterbox_geometry(853, 1280)
    assert (uh + t + b, uw + l + r) == (448, 640) and (uh, uw, t, b, l, r) == (426, 640, 11, 11, 0, 0)
    assert olb.batch_geometry([(853, 1280), (480, 640)]) == (640, 640)  # mixed shapes: auto=False


def test_host_geometry_equals_oracle():
    rng = np.random.default_rng(0)
    for _ in range(500):
        h, w = (int(v) for v in rng.integers(1, 3000, 2))
        for auto in (True, False):
            assert pp.letterbox_geometry(h, w, auto=auto) == olb.letterbox_geometry(h, w, auto=auto), (h, w, auto)


def test_resize_identities():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(olb.resize_linear_u8(img, 37, 53), img)
    const = np.full((31, 47, 3), 173, np.uint8)
    for hw in ((62, 94), (15, 23), (100, 11)):
        assert (olb.resize_linear_u8(const, *hw) == 173).all()


@pytest.mark.parametrize("src,dst", [((40, 60), (80, 120)), ((853, 1280), (426, 640)), ((97, 31), (64, 21))])
def test_resize_matches_torch_bilinear_within_one_level(src, dst):
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, src + (3,), dtype=np.uint8)
    ours = olb.resize_linear_u8(img, *dst).astype(np.int32)
    t = torch.from_numpy(img).permute(2, 0, 1)[None].double()
    ref = F.interpolate(t, size=dst, mode="bilinear", align_corners=False)[0].permute(1, 2, 0).numpy()
    assert np.abs(ours - ref).max() <= 1.0


def test_preprocess_layout():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (853, 1280, 3), dtype=np.uint8)
    x = olb.preprocess([img])
    assert x.shape == (1, 3, 448, 640) and x.dtype == np.float32
    assert np.allclose(x[0, :, :11], 114 / 255) and np.allclose(x[0, :, -11:], 114 / 255)
    lb = olb.letterbox(img)
    assert np.array_equal(x[0, 0], lb[..., 2].astype(np.float32) / np.float32(255))  # RGB plane 0 = BGR channel 2


def test_expand_sources(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(4)
    bgr = rng.integers(0, 256, (21, 34, 3), dtype=np.uint8)
    p = tmp_path / "a.png"
    Image.fromarray(bgr[..., ::-1].copy()).save(p)
    imgs, paths = pp.expand_sources([str(p), bgr, Image.open(p)])
    assert all(np.array_equal(i, bgr) for i in imgs) and paths[0] == str(p)
    imgs, paths = pp.expand_sources(str(tmp_path))
    assert len(imgs) == 1 and np.array_equal(imgs[0], bgr)
    with pytest.raises(FileNotFoundError):
        pp.expand_sources(str(tmp_path / "missing.jpg"))


def test_scale_boxes_equals_oracle():
    from oracle.postprocess import scale_boxes as oscale
    rng = np.random.default_rng(5)
    b = torch.from_numpy(rng.uniform(-20, 660, (50, 4)).astype(np.float32))
    for shape in ((853, 1280), (480, 640), (1000, 700)):
        img1 = olb.batch_geometry([shape])
        assert torch.equal(pp.scale_boxes(img1, b.clone(), shape), oscale(img1, b.clone(), shape))
