#!/bin/bash
# x3 attention with batched loads: x3 GPU tests, per-op tables of yolo11s detect B=8 and yolo11s-seg B=4 (x3).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -2 gpurun_out/x3_tests.log
timeout -k 10 300 python -u tools/op_table.py --model s --dtype x3 > gpurun_out/op_table_s_x3.txt 2>&1 || { tail -20 gpurun_out/op_table_s_x3.txt; exit 1; }
grep -E "attn|total" gpurun_out/op_table_s_x3.txt
timeout -k 10 300 python -u tools/op_table.py --model s --task segment --batch 4 --dtype x3 > gpurun_out/op_table_seg_x3.txt 2>&1 || { tail -20 gpurun_out/op_table_seg_x3.txt; exit 1; }
tail -1 gpurun_out/op_table_seg_x3.txt
