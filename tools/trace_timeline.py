#!/usr/bin/env python3
"""Timeline of graph-replayed forwards from a rocprofv3 --kernel-trace CSV (the bench's prof step).

    python tools/trace_timeline.py <rocprof_dir> [forwards] [skip]

Forwards are split at the input_stats kernel (the first op of every forward).  Per forward: wall span (first start to
last end), the union of kernel-busy intervals (span - union = time no kernel of the forward runs: launch / dependency
gaps), the sum of kernel durations (sum / union > 1: concurrent branches), and the largest idle gaps with the kernels
on either side.  Averaged over the last `forwards` forwards (default 20) before the last `skip` ones (default 0; a
bench.py --steps 50 --warmup 10 run ends with 55 device-loop replays, so skip 55 selects its predict() loop).
"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:\(anonymous namespace\)::|_ZN12_GLOBAL__N_1\d+)?(\w+)", name)
    return (m.group(1) if m else name)[:40]


def main():
    d = sys.argv[1]
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "input_stats" in r[2]]
    fwds = []
    for j in range(len(starts)):
        end = starts[j + 1] if j + 1 < len(starts) else len(rows)
        fwds.append(rows[starts[j]:end])
    fwds = [fw for fw in fwds if len(fw) > 20]
    fwds = fwds[:len(fwds) - skip][-nf:]
    # host bubble: from the last kernel end of a forward to the first kernel start of the next (predict() loops:
    # the counts read, Results, the next call's launch)
    bub = [fwds[j + 1][0][0] - max(e for _, e, _ in fwds[j]) for j in range(len(fwds) - 1)]
    spans, unions, sums, gaps = [], [], [], {}
    for fw in fwds:
        t0 = fw[0][0]
        t1 = max(e for _, e, _ in fw)
        spans.append(t1 - t0)
        sums.append(sum(e - s for s, e, _ in fw))
        u, cur_s, cur_e = 0, None, None
        last = None
        for s, e, n in fw:
            if cur_e is None:
                cur_s, cur_e, last = s, e, n
                continue
            if s > cur_e:
                u += cur_e - cur_s
                key = (short(last), short(n))
                gaps.setdefault(key, []).append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            last = n if e >= cur_e else last
        u += cur_e - cur_s
        unions.append(u)
    k = len(fwds)
    print(f"{k} forwards from {f}")
    print(f"span {sum(spans) / k / 1e3:.1f} us, kernel-busy union {sum(unions) / k / 1e3:.1f} us, "
          f"idle {(sum(spans) - sum(unions)) / k / 1e3:.1f} us, sum of kernel durations {sum(sums) / k / 1e3:.1f} us "
          f"(concurrency {sum(sums) / max(sum(unions), 1):.2f})")
    tot = sorted(((sum(v) / k, len(v) / k, key) for key, v in gaps.items()), reverse=True)
    if bub:
        bs = sorted(bub)
        print(f"between forwards: median {bs[len(bs) // 2] / 1e3:.1f} us, mean {sum(bs) / len(bs) / 1e3:.1f} us")
    tail = {}
    for fw in fwds:  # time of the kernels after the last nms_image (Segment: the mask kernels)
        i = max((k for k, r in enumerate(fw) if "nms_image" in r[2]), default=None)
        if i is not None and i + 1 < len(fw):
            tail.setdefault("after_nms", []).append(max(e for _, e, _ in fw) - fw[i][1])
    if tail:
        v = tail["after_nms"]
        print(f"after the NMS kernel: {sum(v) / len(v) / 1e3:.1f} us per forward (mask kernels)")
    print("largest idle gaps per forward (us, count): after -> before")
    for t, c, (a, b) in tot[:15]:
        print(f"  {t / 1e3:6.2f}  x{c:4.1f}  {a} -> {b}")


if __name__ == "__main__":
    main()
