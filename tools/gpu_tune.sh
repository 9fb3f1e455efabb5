#!/bin/bash
# Re-tune the conv tile tables of the given workloads ("model:task:batch:dtype") on this GPU with per-candidate
# timings (YM_TUNE_LOG), then print the per-op replay table.  New tables land in gpurun_out/tune/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune" YM_TUNE_TABLES=0 YM_TUNE_LOG=1
for w in "$@"; do
  IFS=: read m t b d <<< "$w"
  echo "[tune] $w $(date +%T)"
  timeout -k 10 500 python -u tools/op_table.py --model $m --task $t --batch $b --dtype $d > gpurun_out/tune_${m}_${t}_${b}_${d}.txt 2> gpurun_out/tunelog_${m}_${t}_${b}_${d}.txt || { tail -20 gpurun_out/tunelog_${m}_${t}_${b}_${d}.txt; exit 1; }
  tail -1 gpurun_out/tune_${m}_${t}_${b}_${d}.txt
done
