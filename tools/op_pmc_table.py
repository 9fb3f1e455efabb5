#!/usr/bin/env python3
"""Per-op table of one eager forward from separate rocprofv3 --pmc passes of tools/pmc_forward.py.

    python tools/op_pmc_table.py <ops.txt> <tag> <pmc_dir> [<pmc_dir> ...]

ops.txt is `pmc_forward.py --ops-out` (name, kind, launches, algorithmic FLOPs, algorithmic bytes per op, launch
order).  Counters of an op's launches are summed.  Derived columns (MI355X_MICROARCH.md §rocprofv3 / §DVFS):
  * HBM bytes = FETCH_SIZE x2 + WRITE_SIZE (KiB; the gfx950 half-count of 16 B/lane reads), ratio vs algorithmic;
  * kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs);
  * MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs): the fraction of the chip's MFMA pipe time
    the op kept busy while it ran; achieved TFLOP/s = FLOPs / (kernel cycles / clock), clock = 2.4 GHz nominal.
Writes profiles/<tag>_ops.md and profiles/<tag>_ops.json (its "workload": $YM_OPS_WORKLOAD, the bench.py workload
string bench.py matches to report the time-weighted MFMA busy of the conv family).
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK = 2.4e9


def dispatches(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"kernel": r["Kernel_Name"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    starts = [i for i, e in enumerate(seq) if "input_stats" in e["kernel"]]
    return seq[starts[-1]:]


def short(k):
    k = re.sub(r"^void |\(anonymous namespace\)::|_ZN12_GLOBAL__N_1\d*", "", k)
    return k.split("(")[0][:40]


def main():
    ops_path, tag, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    ops = []
    for ln in open(ops_path):
        if ln.strip():
            name, kind, n, fl, by = ln.rstrip("\n").split("\t")
            ops.append((name, kind, int(n), float(fl), float(by)))
    seqs = [dispatches(d) for d in dirs]
    rows = []
    pos = 0
    for name, kind, n, fl, by in ops:
        c = {}
        kern = None
        for seq in seqs:
            for e in seq[pos:pos + n]:
                kern = kern or short(e["kernel"])
                for k, v in e.items():
                    if k != "kernel":
                        c[k] = c.get(k, 0.0) + v
        pos += n
        r = {"op": name, "kind": kind, "kernel": kern, "flops": fl, "bytes_alg": by}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            r["bytes_pmc"] = 2048 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"]
            r["traffic_ratio"] = r["bytes_pmc"] / by if by else None
        if "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            r["us"] = cyc / CLOCK * 1e6
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                r["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024) if cyc else 0.0
            r["tflops"] = fl / (cyc / CLOCK) / 1e12 if cyc else 0.0
        for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                r[k] = c[k]
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            r["wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        rows.append(r)
    out = os.path.join(ROOT, "profiles", tag)
    json.dump({"sources": [os.path.relpath(d, ROOT) for d in dirs], "clock_hz": CLOCK,
               "workload": os.environ.get("YM_OPS_WORKLOAD"), "ops": rows},
              open(out + "_ops.json", "w"), indent=1)
    conv = [r for r in rows if r["kind"] == "conv"]
    lines = [f"# Per-op PMC table ({tag})", "",
             "One eager forward; columns per MI355X_MICROARCH.md (see tools/op_pmc_table.py). "
             "us from GRBM_GUI_ACTIVE/8 at 2.4 GHz (profiled passes run slightly below nominal clock).", "",
             "| op | kernel | us | TFLOP/s | MFMA busy | alg MB | PMC MB | PMC/alg | wave wait |",
             "|---|---|---|---|---|---|---|---|---|"]
    def f(r, k, fmt):
        v = r.get(k)
        return fmt % v if v is not None else "-"
    for r in rows:
        lines.append(f"| {r['op']} | {r['kernel']} | {f(r, 'us', '%.2f')} | {f(r, 'tflops', '%.0f')} | "
                     f"{f(r, 'mfma_busy', '%.3f')} | {r['bytes_alg'] / 1e6:.2f} | "
                     f"{(r['bytes_pmc'] / 1e6) if 'bytes_pmc' in r else float('nan'):.2f} | {f(r, 'traffic_ratio', '%.2f')} | "
                     f"{f(r, 'wait_frac', '%.2f')} |")
    tot = {k: sum(r.get(k, 0.0) or 0.0 for r in conv) for k in ("us", "flops", "bytes_alg", "bytes_pmc")}
    if tot["bytes_alg"]:
        lines += ["", f"conv HBM bytes (PMC) / algorithmic: {tot['bytes_pmc'] / tot['bytes_alg']:.3f} "
                      f"({tot['bytes_pmc'] / 1e6:.1f} / {tot['bytes_alg'] / 1e6:.1f} MB per forward)"]
    if tot["us"]:
        busy = sum((r.get("mfma_busy", 0.0) or 0.0) * r.get("us", 0.0) for r in conv) / tot["us"]
        lines += ["", f"conv total: {tot['us']:.1f} us, {tot['flops'] / (tot['us'] * 1e-6) / 1e12:.0f} TFLOP/s, "
                      f"MFMA busy (time-weighted) {busy:.3f}, PMC/alg bytes "
                      f"{(tot['bytes_pmc'] / tot['bytes_alg']) if tot['bytes_alg'] else 0:.3f}"]
    open(out + "_ops.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-3:]))


if __name__ == "__main__":
    main()
