"""Multi-rank plumbing on CPU with gloo (world_size 2): the init-time model-blob broadcast is byte-exact on every
rank and batch shards tile the global batch.  On MI355X the same code runs over RCCL (backend 'nccl')."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from yolomi.dist import broadcast_blob, digest, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = None
        if rank == 0:
            from yolomi.plan import pack_model
            from yolomi.synth import synth_weights
            blob = pack_model("n", "detect", synth_weights("n", "detect", 0), "f16")
        got = broadcast_blob(blob, torch.device("cpu"))
        h = torch.tensor(list(bytes.fromhex(digest(got))), dtype=torch.uint8)
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        q.put((rank, len(got), all(torch.equal(hs[0], x) for x in hs), shard(8 * world, rank, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_blob_broadcast_and_shards_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, _free_port() if r < 0 else PORT, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == res[1][1] > 1_000_000
    assert all(r[2] for r in res)
    assert [r[3] for r in res] == [(0, 8), (8, 16)]


PORT = _free_port()


def test_shard_ranges():
    for gb, w in ((8, 1), (16, 2), (17, 4), (3, 8)):
        spans = [shard(gb, r, w) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == gb
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1
    with pytest.raises(ValueError):
        shard(8, 2, 2)


@pytest.mark.timeout(300)
def test_bench_spawns_its_own_ranks_plumbing_world2():
    """`bench.py --gpus 2` without a launcher starts the two ranks itself (torch.distributed.run as a child); the
    CPU/gloo rehearsal of its protocol reports n_gpus = 2, identical blobs on every rank and the /255 statistic
    all-reduced over the global batch every step (only the last rank holds a 0-255 image)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing", "--model", "n",
                        "--steps", "5", "--warmup", "1"], capture_output=True, text=True, timeout=280, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["blob_equal_on_all_ranks"] and d["blob_bytes"] > 1_000_000
    assert d["global_batch_max"] > 200.0
    # verdict r5 item 7: the N > 1 step reads its shard for the /255 rule every step, as N = 1's forward does
    assert d["batch_max_reads_per_step"] == 1.0 and d["batch_rule"].startswith("per step")


def test_bench_refuses_mislabelled_world():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.gpu
def test_rccl_cabi_broadcast_two_ranks():
    """ym_broadcast_weights with a receiving rank: rank 1's empty context gets rank 0's blob over RCCL
    and both compute the same detections.  Ranks go to separate GPUs when the box has two; on a one-GPU box both
    share GPU 0 where RCCL allows it (its duplicate-GPU check may refuse: then skipped)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = 29500 + (os.getpid() % 2000)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               NCCL_DEBUG="WARN")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(root, "tools", "rccl_bcast_check.py")],
                       capture_output=True, text=True, timeout=240, env=env)
    out = p.stdout + p.stderr
    one_gpu = torch.cuda.device_count() < 2
    if p.returncode != 0 and one_gpu and ("uplicate GPU" in out or "invalid usage" in out):
        pytest.skip("RCCL refuses two ranks on one GPU (ncclCommInitRank: invalid usage)")
    assert p.returncode == 0, out[-3000:]
    assert "digests equal: True" in out
