#!/usr/bin/env python3
"""Median nms_image / decode_anchors kernel times per confidence of tools/nms_probe.py from its rocprofv3 trace.
    python tools/nms_summary.py gpurun_out/nmsp"""
import csv, glob, os, statistics, sys
rows = list(csv.DictReader(open(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0])))
def times(pat):
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if pat in r["Kernel_Name"]]
nms, dec = times("nms_image"), times("decode_anchors")
confs = [float(c) for c in os.environ.get("NMS_CONFS", "0.99,0.5,0.25,0.1").split(",")]
per = len(nms) // len(confs)
for i, c in enumerate(confs):
    print(f"conf {c}: nms {statistics.median(nms[i * per:(i + 1) * per]):.1f} us, "
          f"decode {statistics.median(dec[i * per:(i + 1) * per]):.1f} us")
