#!/bin/bash
# Per-op replay tables (tools/op_table.py) for the given workloads: "model:task:batch:dtype" ...
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for w in "$@"; do
  IFS=: read m t b d <<< "$w"
  echo "[optable] $w $(date +%T)"
  timeout -k 10 300 python -u tools/op_table.py --model $m --task $t --batch $b --dtype $d > gpurun_out/optable_${m}_${t}_${b}_${d}.txt 2>&1 || { tail -20 gpurun_out/optable_${m}_${t}_${b}_${d}.txt; exit 1; }
done
