"""The receive path of the init-time weight broadcast on one GPU (SURVEY §4.4's fake backend).

`ym_broadcast_weights_local` runs the per-rank steps of `ym_broadcast_weights` — staging buffer, the root's upload,
a receiver's copy-out, `ym_load_weights`, the verdict every rank agrees on (csrc/ym_runtime.cpp BcastRank) — with
the ranks as contexts of this process and device-to-device copies where RCCL would move the chunks.  So the code
that the RCCL transport's non-root ranks run executes here on a one-GPU box."""
import pytest
import torch

from tests.golden.make_golden import make_input
from yolomi.lib import Runtime, YMError
from yolomi.plan import pack_model
from yolomi.synth import synth_weights

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _make(scale, dtype):
    from core.model import YOLO11Model

    def make(**kw):
        return YOLO11Model(task="detect", size=scale, device="cuda:0", dtype=dtype, verbose=False, **kw)
    return make


@pytest.mark.parametrize("dtype", ["x3", "f16"])
def test_local_broadcast_receivers_match_root(dtype):
    """Three 'ranks' on GPU 0: ranks 1 and 2 start empty, receive rank 0's blob and produce bit-identical
    detection rows on the same batch (blob > one 16 MB staging chunk for yolo11s x3: the chunk loop runs twice)."""
    from yolomi.dist import local_broadcast_models
    scale = "s" if dtype == "x3" else "n"
    blob = pack_model(scale, "detect", synth_weights(scale, "detect", 0), dtype)
    if dtype == "x3":
        assert len(blob) > 16 << 20
    models = local_broadcast_models(_make(scale, dtype), blob, 3, DEV, root=0, scale=scale, task="detect",
                                    dtype=dtype)
    x = make_input("uniform", (41, 42), 640).to(DEV)
    rows = []
    for m in models:
        rows.append([r.boxes.data.clone() for r in m.predict(x, conf=0.1)])
    assert sum(len(r) for r in rows[0]) > 10
    for other in rows[1:]:
        for a, b in zip(rows[0], other):
            assert torch.equal(a, b)


def test_local_broadcast_failures_return_one_verdict():
    """No weights on the root: every rank fails before the transfer.  A receiver whose context was created for
    another plan (dtype mismatch): its ym_load_weights fails, the call reports it, the other receiver still loads."""
    blob = pack_model("n", "detect", synth_weights("n", "detect", 0), "f16")
    stream = torch.cuda.current_stream(DEV).cuda_stream
    empty = [Runtime(0, None, scale="n", task="detect", dtype="f16") for _ in range(2)]
    with pytest.raises(YMError, match="no weights to broadcast"):
        Runtime.broadcast_weights_local(empty, 0, stream)
    root = Runtime(0, blob, scale="n", task="detect", dtype="f16")
    good = Runtime(0, None, scale="n", task="detect", dtype="f16")
    wrong = Runtime(0, None, scale="n", task="detect", dtype="x3")
    with pytest.raises(YMError):
        Runtime.broadcast_weights_local([root, good, wrong], 0, stream)
    assert good.lib.ym_num_ops(good.ctx) == root.n_ops  # the matching receiver did load the blob
    with pytest.raises(YMError, match="out of range"):
        Runtime.broadcast_weights_local([root, good], 2, stream)
