#!/usr/bin/env python3
"""Carry the committed conv tables over a plan change (ops renamed, merged or removed, e.g. GraphBuilder.fuse_dw):
an op whose name survives keeps its committed (in-context refined) cfg, an op the old table does not name takes the
pick of a fresh ym_tune on this GPU.  Writes gpurun_out/tuned/<table>.json (copy into yolomi/tuned/ to commit).

    python tools/retable.py [scale:task:dtype:B ...]     (default: the committed x3 tables)
YM_RETABLE_OPS=a,b: ops whose committed cfg is replaced by the fresh tune's pick too."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)
os.environ["YM_TUNE_TABLES"] = "0"  # ignore every table: the engine runs ym_tune on first use
import torch  # noqa: E402

from bench import synthetic_batch  # noqa: E402
from core.model import YOLO11Model  # noqa: E402
from yolomi.engine import TUNE_VERSION, TUNED_DIR  # noqa: E402

specs = sys.argv[1:] or ["s:detect:x3:8", "n:detect:x3:8", "s:segment:x3:4"]
out_dir = os.path.join(ROOT, "gpurun_out", "tuned")
os.makedirs(out_dir, exist_ok=True)
dev = torch.device("cuda", 0)
for spec in specs:
    scale, task, dtype, B = spec.split(":")
    B = int(B)
    m = YOLO11Model(task=task, size=scale, device="cuda:0", dtype=dtype, verbose=False)
    eng = m.model.engine
    name = eng._table_name(B, 640, 640)
    try:
        old = json.load(open(os.path.join(TUNED_DIR, name)))
    except OSError:
        old = {"ops": [], "cfg": []}
    # YM_RETABLE_OPS: op names to re-tune as well (a kernel family gained a configuration for them)
    retune = set(filter(None, os.environ.get("YM_RETABLE_OPS", "").split(",")))
    keep = {n: c for n, c in zip(old["ops"], old["cfg"]) if n not in retune}
    eng.run(synthetic_batch(B, 640, 1000, dev))  # tunes (no table)
    torch.cuda.synchronize()
    tuned = eng.rt.get_op_cfg(B, 640, 640)
    ops = [op.name for op in eng.graph.ops]
    cfg = [keep.get(n, t) for n, t in zip(ops, tuned)]
    new = [n for n in ops if n not in keep]
    table = {"version": TUNE_VERSION, "device": torch.cuda.get_device_properties(dev).gcnArchName,
             "ncfg": eng._ncfg(), "ops": ops, "cfg": cfg,
             "note": (old.get("note", "") + f"; carried over a plan change by tools/retable.py (new ops from ym_tune: "
                      f"{', '.join(new)})").lstrip("; ")}
    json.dump(table, open(os.path.join(out_dir, name), "w"))
    print(f"{name}: {len(ops)} ops, {len(new)} new: " + ", ".join(f"{n}={c}" for n, c in zip(ops, cfg) if n in new),
          flush=True)
