#!/bin/bash
# Round-5 A/B: the 4-stream branch schedule (YM_BRANCHES=4) against the serial order (1) on the plans that run serially
# by default (int8 / fp8 PTQ, yolo11n B=8; the segment plan, yolo11s-seg B=4 x3) — round 2 measured it 12-15 % slower
# there; the kernels have changed since.  Bench lines without the CPU leg, each variant twice, interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05f}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/steps.log"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
for rep in 1 2; do
  for br in 1 4; do
    YM_BRANCHES=$br run "i8_br${br}_$rep" 400 python -u bench.py --model n --dtype i8 --steps 50 --warmup 10 --no-cpu --no-roofline
    YM_BRANCHES=$br run "f8_br${br}_$rep" 400 python -u bench.py --model n --dtype f8 --steps 50 --warmup 10 --no-cpu --no-roofline
    YM_BRANCHES=$br run "seg_br${br}_$rep" 400 python -u bench.py --task segment --batch 4 --steps 50 --warmup 10 --no-cpu --no-roofline --no-f16
  done
done
echo done >> "$OUT/steps.log"
