#!/usr/bin/env python3
"""Per-op replay time of one model at several batch sizes (each autotuned on this GPU): does a layer's time grow with
its work (throughput-bound kernel) or stay flat (latency / launch bound)?  Prints one JSON object.

    python tools/batch_scaling.py [--model s] [--batches 8,16,32] [--out gpurun_out/scaling.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="s")
    ap.add_argument("--batches", default="8,16,32")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from bench import synthetic_batch
    from core.model import YOLO11Model
    m = YOLO11Model(task="detect", size=a.model, device="cuda:0", dtype="f16")
    eng = m.model.engine
    res = {"model": a.model, "ops": [op.name for op in eng.graph.ops], "batches": {}}
    for B in [int(b) for b in a.batches.split(",")]:
        t0 = time.time()
        x = synthetic_batch(B, a.size, 1000, torch.device("cuda", 0))
        eng.run(x)
        torch.cuda.synchronize()
        t = eng.profile_replay(x, reps=20)
        # whole-forward graph replay time
        for _ in range(3):
            eng.run(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            eng.run(x)
        e1.record()
        torch.cuda.synchronize()
        costs = eng.graph.op_costs(B, a.size, a.size, 2)
        res["batches"][B] = {"op_ms": list(t), "flops": [c[0] for c in costs], "bytes": [c[1] for c in costs],
                             "forward_ms": e0.elapsed_time(e1) / 20, "tune_source": str(eng.tune_source.get((B, a.size, a.size))),
                             "setup_s": time.time() - t0}
        print(f"B={B}: forward {res['batches'][B]['forward_ms']:.3f} ms, sum ops {sum(v for v in t if v > 0):.3f} ms",
              flush=True)
    bs = sorted(res["batches"])
    print(f"{'op':28s}" + "".join(f"{'B=' + str(b):>10s}" for b in bs))
    for i, name in enumerate(res["ops"]):
        row = [res["batches"][b]["op_ms"][i] for b in bs]
        if row[0] < 0:
            continue
        print(f"{name:28s}" + "".join(f"{v * 1e3:10.1f}" for v in row))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
