#!/bin/bash
# Round-3 batch: NMS phase ablation, x3 lanes / branch-stream A/B, in-context refinement of the x3 yolo11s B=8 table.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
for d in 0 1 2 3 4 5 7; do
  YM_NMS_DBG=$d timeout -k 10 120 python -u tools/nms_phases.py >> gpurun_out/nms_phases.txt 2>> gpurun_out/nms_phases.err || { tail -20 gpurun_out/nms_phases.err; exit 1; }
done
cat gpurun_out/nms_phases.txt
bash tools/gpu_lanes_ab.sh || exit 1
bash tools/gpu_ctx_refine.sh s detect 8 3 x3 || exit 1
