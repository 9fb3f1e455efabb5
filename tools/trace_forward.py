#!/usr/bin/env python3
"""One graph-replayed forward from a rocprofv3 --kernel-trace CSV, kernel by kernel: start offset, duration, queue,
and what it waited for — the previous kernel on its own queue, or (a cross-queue join) a kernel on another queue that
ended shortly before it started.  Locates the ~10 us join gaps of the branch schedule (tools/trace_timeline.py counts
them).

    python tools/trace_forward.py <rocprof_dir> [forward index from the end of the predict loop, default 30]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::|_ZN12_GLOBAL__N_1\d+)?(\w+)(<[^(]*>)?", name)
    return ((m.group(1) + (m.group(2) or "")) if m else name)[:70]


def main():
    d = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"],
                     int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "input_stats" in r[3]]
    # the predict loop's forwards are followed by the bench's device loop (55 replays) and the eager profiles
    k = starts[max(0, len(starts) - 55 - back)]
    k2 = starts[starts.index(k) + 1]
    fw = rows[k:k2]
    t0 = fw[0][0]
    last_end = {}
    print(f"forward of {len(fw)} kernels, span {(max(r[1] for r in fw) - t0) / 1e3:.1f} us")
    print(f"{'start':>8} {'dur':>6} {'q':>2} {'gap':>6}  {'waited for':32s} kernel (grid/wg)")
    for s, e, q, name, gx, wx in fw:
        prev_q = last_end.get(q)
        # the latest-ending kernel on another queue that ended before this start
        other = max(((r[1], r) for r in fw if r[2] != q and r[1] <= s), default=(None, None))[1]
        cause = ""
        gap = (s - prev_q[1]) / 1e3 if prev_q else 0.0
        if other is not None and (prev_q is None or other[1] > prev_q[1]) and (s - other[1]) < 20000:
            cause = f"q{other[2]} {short(other[3])[:28]}"
            gap = (s - other[1]) / 1e3
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:6.1f} {q:2d} {gap:6.1f}  {cause:32s} {short(name)} ({gx // max(wx, 1)}/{wx})")
        last_end[q] = (s, e)


if __name__ == "__main__":
    main()
