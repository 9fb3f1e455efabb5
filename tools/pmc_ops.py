#!/usr/bin/env python3
"""Per-op PMC counters of one eager forward: joins rocprofv3 --pmc counter_collection.csv dispatches (last forward,
split at input_stats) with the op list written by `tools/pmc_forward.py --ops-out`.

    python tools/pmc_ops.py <ops.txt> <pmc_dir> [<pmc_dir> ...] [--ops regex]

SQ_* wave counters count quad-cycles (MI355X_MICROARCH.md §Per-instruction cycle constants); printed per wave.
"""
import csv
import glob
import os
import re
import sys


def last_forward(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": r["Kernel_Name"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    starts = [i for i, e in enumerate(seq) if "input_stats" in e["name"]]
    return seq[starts[-1]:]


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    pat = re.compile(sys.argv[sys.argv.index("--ops") + 1]) if "--ops" in sys.argv else None
    if pat:
        args.remove(pat.pattern)
    ops = [ln.rstrip("\n").split("\t") for ln in open(args[0]) if ln.strip()]
    ops = [o for o in ops if o[1] != "input"]
    fwd = None
    for d in args[1:]:
        seq = last_forward(d)[1:]  # input_stats = the input op
        if fwd is None:
            fwd = seq
        else:
            for a, b in zip(fwd, seq):
                a.update({k: v for k, v in b.items() if k != "name"})
    cols = sorted({k for e in fwd for k in e if k != "name"})
    print(f"{'op':24s} {'kernel':28s} " + " ".join(f"{c[:14]:>14s}" for c in cols))
    for (name, kind), e in zip(ops, fwd):
        if pat and not pat.search(name):
            continue
        kn = re.sub(r"^void |\(anonymous namespace\)::|_ZN12_GLOBAL__N_1\d*", "", e["name"])[:28]
        print(f"{name:24s} {kn:28s} " + " ".join(f"{e.get(c, 0):14.0f}" for c in cols))


if __name__ == "__main__":
    main()
