#!/usr/bin/env python3
"""Markdown table of bench.py lines: python tools/bench_table.py profiles/r03e_bench_*.json"""
import json
import sys


def main():
    print("| workload | plan | images/s (predict loop) | device images/s | conv TFLOP/s (frac, isolated replay) | "
          "frac under the real schedule (rocprof) | per-launch roofline frac | parity vs CPU oracle | CPU oracle img/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        d = json.load(open(p))
        r = d.get("roofline", {})
        par = d.get("parity")
        acc = d.get("accuracy", {})
        if par:
            pv = (f"meets 7-1(b): max \\|Δxy\\| {par['max_dxy_px']} px, \\|Δscore\\| {par['max_dscore']}"
                  if par["meets_tolerance"] else f"misses 7-1(b): \\|Δscore\\| {par['max_dscore']}")
        elif acc:
            pv = f"mAP50-95 {acc.get('map50_95')} vs {acc.get('gt', '')[:24]}"
        else:
            pv = "—"
        cpu = d.get("cpu_baseline", {}).get("value", "—")
        unit = "TOP/s" if d["dtype"] == "i8" else "TFLOP/s"
        print(f"| {d['config']['workload'].split(',')[0]} | {d['dtype']} | **{d['value']:,.0f}** | "
              f"{d['device_images_per_s']:,.0f} | {r.get('achieved', '—')} {unit} ({r.get('frac', '—')}) | "
              f"{r.get('frac_rocprof', '—')} | {r.get('per_launch_roofline_frac', '—')} | {pv} | {cpu} |")


if __name__ == "__main__":
    main()
