"""Per-op device-time table of one forward (HIP events around every launch, eager) with GEMM shape, algorithmic
FLOPs/bytes and achieved TFLOP/s / GB/s.

    python -m yolomi.profile --model n --batch 8 --size 640 [--dtype f16] [--reps 10]
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import torch


KERNELS_PER_OP = {"input": 1}


def trace_times(csv_path: str, n_ops_kernels: int, kinds):
    """Kernel durations (ms) per plan op from a rocprofv3 --kernel-trace CSV: the LAST complete forward's dispatches
    in order (every op = 1 kernel: the input op is input_stats)."""
    import csv
    rows = list(csv.DictReader(open(csv_path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # forwards start with the init kernel of the input op
    starts = [i for i, n in enumerate(names) if "input_stats" in n]
    s = starts[-1]
    seg = rows[s:s + n_ops_kernels]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in seg]
    wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) * 1e-6
    out, k = [], 0
    for kind in kinds:
        nk = KERNELS_PER_OP.get(kind, 1)
        out.append(sum(durs[k:k + nk]))
        k += nk
    return np.array(out), wall, [r["Kernel_Name"] for r in seg]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="n")
    ap.add_argument("--task", default="detect")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default="f16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--top", type=int, default=200)
    ap.add_argument("--trace", default="", help="rocprofv3 kernel_trace.csv of a previous `--replay` run")
    ap.add_argument("--replay", action="store_true", help="only run graph replays (for rocprofv3 --kernel-trace)")
    a = ap.parse_args(argv)
    from .arch import GraphBuilder
    B, S = a.batch, a.size
    if a.trace:
        g = GraphBuilder(a.model, a.task)
        kinds = [op.kind for op in g.ops]
        nk = sum(KERNELS_PER_OP.get(k, 1) for k in kinds)
        t, wall, _ = trace_times(a.trace, nk, kinds)
        print(f"trace: last forward first-dispatch → last-end wall {wall:.4f} ms, kernel sum {t.sum():.4f} ms")
        _table(g, t, B, S, a)
        return
    from .engine import Engine
    from .synth import synth_weights, uniform
    dev = torch.device("cuda", 0)
    eng = Engine(a.model, a.task, synth_weights(a.model, a.task, 0), dev, a.dtype)
    x = torch.from_numpy(uniform(5, B * 3 * S * S).astype(np.float32).reshape(B, 3, S, S)).to(dev)
    if a.replay:
        for _ in range(a.reps):
            eng.run(x)
        torch.cuda.synchronize()
        return
    eng.run(x)
    eng.profile(x)
    t = np.zeros(len(eng.graph.ops))
    for _ in range(a.reps):
        t += np.array(eng.profile(x))
    t /= a.reps
    _table(eng.graph, t, B, S, a)


def _table(graph, t, B, S, a):
    class _E:
        pass
    eng = _E()
    eng.graph = graph
    costs = eng.graph.op_costs(B, S, S, 2 if a.dtype == "f16" else 4)
    rows = []
    for i, op in enumerate(eng.graph.ops):
        ar = op.args
        shape = ""
        if op.kind == "conv":
            fo = eng.graph.out_factor(op)
            M = B * (S // fo) ** 2
            shape = f"k{ar['k']}s{ar['s']} M={M} N={ar['c2']} K={ar['k'] ** 2 * ar['c1']}"
        fl, by = costs[i]
        ms = t[i]
        rows.append((ms, op.kind, op.name, shape, fl / (ms * 1e-3) / 1e12 if ms > 0 else 0,
                     by / (ms * 1e-3) / 1e9 if ms > 0 else 0))
    print(f"yolo11{a.model} {a.task} B={B} {S}x{S} {a.dtype}: eager op sum {t.sum():.3f} ms, "
          f"{len(rows)} ops", flush=True)
    print(f"{'ms':>8} {'kind':>6} {'TF/s':>7} {'GB/s':>7}  name  shape")
    for r in sorted(rows, reverse=True)[: a.top]:
        print(f"{r[0]:8.4f} {r[1]:>6} {r[4]:7.1f} {r[5]:7.0f}  {r[2]}  {r[3]}")
    kinds = {}
    for r in rows:
        kinds[r[1]] = kinds.get(r[1], 0) + r[0]
    print("by kind:", {k: round(v, 4) for k, v in kinds.items()})


if __name__ == "__main__":
    sys.exit(main())
