#!/bin/bash
# Round-5 check of the yolo11s-seg B=4 predict() loop (r05f's 50-step lines read 1.75-2.09k img/s against 2.5k in
# round 4 at 200 steps): the bench at the round-4 length, twice, and tools/seg_host.py's per-step split.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05j}
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
for step in ${STEPS:-seg host}; do
  case $step in
    seg) for rep in 1 2; do
           run "bench_seg_$rep" 400 python -u bench.py --task segment --batch 4 --steps 200 --warmup 20 --no-cpu --no-roofline --no-f16
         done ;;
    host) run seg_host 300 python -u tools/seg_host.py s ;;
  esac
done
echo done >> "$OUT/steps.log"
