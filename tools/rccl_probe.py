"""One-rank RCCL bootstrap through the C-ABI (ym_rccl_get_unique_id / ym_rccl_comm_init / ym_broadcast_weights)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
import torch  # noqa: E402,F401
from yolomi import lib as L  # noqa: E402
from yolomi.plan import pack_model  # noqa: E402
from yolomi.synth import synth_weights  # noqa: E402

uid = L.rccl_unique_id()
print("uid ok", uid[:8].hex(), flush=True)
comm = L.rccl_comm_init(0, 1, uid, 0)
print("comm ok", hex(comm), flush=True)
rt = L.Runtime(0, pack_model("n", "detect", synth_weights("n", "detect", 0), "f16"))
rt.broadcast_weights(comm, 0, 0)
print("broadcast ok", flush=True)
L.rccl_comm_destroy(comm)
