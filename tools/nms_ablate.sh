#!/bin/bash
# NMS phase ablation (YM_NMS_DBG = exit after phase k of the bit-matrix path; timing only): nms_image average
# duration per value, from rocprofv3 --kernel-trace --stats over eager forwards of the s B=8 bench workload.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
for d in ${DBGS:-0 1 2 3 4 5 6 7}; do
  rm -rf gpurun_out/nms_ab_$d
  (cd /tmp && YM_NMS_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/nms_ab_$d" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model ${1:-s} --reps 20 > "$R/gpurun_out/nms_ab_$d.log" 2>&1) || exit 1
  echo "dbg=$d $(grep -E 'nms_image|decode_anchors' gpurun_out/nms_ab_$d/run_kernel_stats.csv | cut -d, -f1,2,4 | tr '\n' ' ')"
done
