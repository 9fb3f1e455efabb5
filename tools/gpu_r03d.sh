#!/bin/bash
# Round-3 batch: NMS phase ablation, x3 lanes / branch-stream A/B, in-context refinement of the x3 yolo11s B=8 table.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -2 gpurun_out/x3_tests.log
for m in s n; do
  timeout -k 10 300 python -u tools/op_table.py --model $m --dtype x3 > gpurun_out/op_table_${m}_x3.txt 2>&1 || { tail -20 gpurun_out/op_table_${m}_x3.txt; exit 1; }
  tail -1 gpurun_out/op_table_${m}_x3.txt
done
for d in 0 1 2 3 4 5 7; do
  YM_NMS_DBG=$d timeout -k 10 120 python -u tools/nms_phases.py >> gpurun_out/nms_phases.txt 2>> gpurun_out/nms_phases.err || { tail -20 gpurun_out/nms_phases.err; exit 1; }
done
cat gpurun_out/nms_phases.txt
for t in 0 1 2 3; do
  YM_DW_TILE=$t timeout -k 10 200 python -u tools/op_table.py --model s --dtype x3 > gpurun_out/dwtile_$t.txt 2>&1 || { tail -20 gpurun_out/dwtile_$t.txt; exit 1; }
  echo "dw tile $t"; grep -E "dwconv" gpurun_out/dwtile_$t.txt
done
bash tools/gpu_lanes_ab.sh || exit 1
bash tools/gpu_ctx_refine.sh s detect 8 3 x3 || exit 1
