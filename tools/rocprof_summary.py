#!/usr/bin/env python3
"""Turn rocprofv3 output into the per-round evidence committed under profiles/.

    python tools/rocprof_summary.py stats  <rocprof_dir> <tag> [workload description]   # --stats run of bench.py
    python tools/rocprof_summary.py pmc    <fetch_dir> <write_dir> <tag> [workload description]

`stats`: copies kernel_stats.csv to profiles/<tag>_kernel_stats.csv and writes profiles/<tag>_summary.json with the
conv implicit-GEMM family time per forward (forwards counted by stem-kernel dispatches) — the figure bench.py's
live HIP-event roofline must agree with.
`pmc`: per-forward FETCH_SIZE / WRITE_SIZE of the conv family from two separate --pmc passes of
tools/pmc_forward.py, corrected as MI355X_MICROARCH.md §HBM prescribes (gfx950 FETCH_SIZE counts half the bytes of
wide coalesced 16 B/lane reads → ×2; WRITE_SIZE exact for 16 B/lane stores); rocprofv3 reports both in KiB.
Writes profiles/<tag>_pmc.json, which bench.py reads for roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
CONV = re.compile(r"conv_igemm|conv_lds|conv_dma|conv_i8|conv_stream|conv_small|conv_halo|conv_bneck|conv_dwpw")
STEM = re.compile(r"stem_conv3x3s2|stem_i8|stem_mfma|stem_valu")
CALIB = re.compile(r"conv_igemm<float, float|conv_igemmIffL")  # the f32 calibration forwards of an int8 run


def family(name):
    if CALIB.search(name):
        return "calib_f32_conv"
    if STEM.search(name):
        return "stem"
    if CONV.search(name):
        return "conv"
    for k in ("dwconv3x3", "sppf", "attn_psa", "decode_anchors", "nms_image", "input_stats", "spin_wait", "requant_copy",
              "copyBuffer"):
        if k in name:
            return k
    return "other"


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def stats(d, tag, workload=None):
    ks = find(d, "kernel_stats.csv")
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(ks, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(ks)))
    fam = {}
    for r in rows:
        f = family(r["Name"])
        e = fam.setdefault(f, {"calls": 0, "total_ns": 0.0})
        e["calls"] += int(r["Calls"])
        e["total_ns"] += float(r["TotalDurationNs"])
    nfwd = fam.get("stem", {}).get("calls", 0)
    out = {"source": os.path.relpath(ks, ROOT), "workload": workload, "forwards": nfwd, "families": {}}
    for f, e in sorted(fam.items(), key=lambda kv: -kv[1]["total_ns"]):
        out["families"][f] = {"calls": e["calls"], "total_ms": round(e["total_ns"] / 1e6, 3),
                              "avg_us": round(e["total_ns"] / e["calls"] / 1e3, 3),
                              "ms_per_forward": round(e["total_ns"] / max(nfwd, 1) / 1e6, 4)}
    json.dump(out, open(os.path.join(PROF, f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


def pmc_per_forward(d, counter, reps):
    rows = list(csv.DictReader(open(find(d, "counter_collection.csv"))))
    disp = {}
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, [r["Kernel_Name"], 0.0])
        e[1] += float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    starts = [i for i, (n, _) in enumerate(seq) if "input_stats" in n]
    if len(starts) < reps:
        raise SystemExit(f"{d}: found {len(starts)} forwards, need {reps}")
    fwd = []
    for j in range(len(starts) - reps, len(starts)):
        end = starts[j + 1] if j + 1 < len(starts) else len(seq)
        per = {}
        for n, v in seq[starts[j]:end]:
            per[family(n)] = per.get(family(n), 0.0) + v
        fwd.append(per)
    keys = set().union(*fwd)
    return {k: sum(p.get(k, 0.0) for p in fwd) / reps for k in keys}


def pmc(fetch_dir, write_dir, tag, reps=3, workload=None):
    fe = pmc_per_forward(fetch_dir, "FETCH_SIZE", reps)
    wr = pmc_per_forward(write_dir, "WRITE_SIZE", reps)
    fams = sorted(set(fe) | set(wr))
    per = {f: {"fetch_kib_raw": round(fe.get(f, 0.0), 1), "write_kib": round(wr.get(f, 0.0), 1),
               "bytes_corrected": int(2 * fe.get(f, 0.0) * 1024 + wr.get(f, 0.0) * 1024)} for f in fams}
    out = {"workload": workload, "forwards_averaged": reps, "unit": "bytes per forward (all launches of the family)",
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16B/lane reads), WRITE_SIZE x1; KiB -> bytes",
           "families": per}
    for d in (fetch_dir, write_dir):
        dst = os.path.join(PROF, f"{tag}_{os.path.basename(os.path.normpath(d))}_counter_collection.csv")
        shutil.copy(find(d, "counter_collection.csv"), dst)
    json.dump(out, open(os.path.join(PROF, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3], workload=sys.argv[4] if len(sys.argv) > 4 else None)
    elif sys.argv[1] == "pmc":
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], workload=sys.argv[5] if len(sys.argv) > 5 else None)
    else:
        raise SystemExit(__doc__)
