#!/bin/bash
# Same-box A/B of environment settings on one bench command, alternating A B A B (each arm its own limit).
#   TAG=r06o ARGS="--model n --dtype i8 --no-cpu" A="YM_BRANCHES=1" B="YM_BRANCHES=4" bash tools/gpu_ab_env.sh
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for arm in A B A B; do
  n=$((n + 1))
  env ${!arm} timeout -k 10 300 python -u bench.py --no-roofline --steps ${STEPS:-300} $ARGS > "$OUT/ab_${arm}_$n.log" 2>&1
  rc=$?
  echo "[$arm ${!arm}] rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
