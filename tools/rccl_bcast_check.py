#!/usr/bin/env python3
"""Two-or-more-rank check of the C-ABI weight broadcast (ym_broadcast_weights via yolomi.dist.rccl_broadcast_model):
rank 0 packs the blob, every other rank's context receives it over RCCL; each rank then runs the same batch and the
ranks compare detection digests (run under torch.distributed.run; tests/test_dist.py).  The RCCL unique id travels
over a gloo group, so the ranks may share one GPU where RCCL allows it."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from bench import synthetic_batch
    from core.model import YOLO11Model
    from yolomi.dist import rccl_broadcast_model
    from yolomi.plan import pack_model
    from yolomi.synth import synth_weights
    blob = pack_model("n", "detect", synth_weights("n", "detect", 0), "f16") if rank == 0 else None

    def make(**kw):
        return YOLO11Model(task="detect", size="n", device=str(dev), dtype="f16", verbose=False, **kw)
    m = rccl_broadcast_model(make, blob, dev)
    x = synthetic_batch(2, 320, 77, dev)
    d, c = m.model.engine.run(x, conf=0.1)
    dets = torch.cat([d[b, :int(c[b])] for b in range(2)]).cpu().numpy().tobytes()
    h = hashlib.sha256(dets).hexdigest()
    hs = [None] * world
    dist.all_gather_object(hs, h)
    if rank == 0:
        print(f"rccl_bcast_check: world {world} on {ngpu} GPU(s), digests equal: {len(set(hs)) == 1}, "
              f"dets bytes {len(dets)}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if len(set(hs)) == 1 else 3)


if __name__ == "__main__":
    main()
