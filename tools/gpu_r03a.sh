#!/bin/bash
# Round-3 probe: depthwise strip-variant tests, per-op replay tables of the x3 plan (strip dw on / off), yolo11s B=8.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread > gpurun_out/kern_tests.log 2>&1 || { tail -30 gpurun_out/kern_tests.log; exit 1; }
tail -3 gpurun_out/kern_tests.log
for d in x3 f16; do
  timeout -k 10 300 python -u tools/op_table.py --model s --dtype $d > gpurun_out/op_table_s_$d.txt 2>&1 || { tail -20 gpurun_out/op_table_s_$d.txt; exit 1; }
  tail -2 gpurun_out/op_table_s_$d.txt
  YM_DW_RT=1 timeout -k 10 300 python -u tools/op_table.py --model s --dtype $d > gpurun_out/op_table_s_${d}_rt1.txt 2>&1 || { tail -20 gpurun_out/op_table_s_${d}_rt1.txt; exit 1; }
  grep -E "dw|total|sum" gpurun_out/op_table_s_${d}_rt1.txt | tail -8
  grep -E "dw" gpurun_out/op_table_s_$d.txt
done
