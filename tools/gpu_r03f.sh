#!/bin/bash
# Round-3 batch: branch-stream A/B of the x3 segment plan (yolo11s-seg B=4), in-context refinement of the x3 yolo11n
# B=8 table.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
for rep in 1 2; do
  for br in 1 4; do
    YM_BRANCHES=$br timeout -k 10 200 python bench.py --task segment --batch 4 --dtype x3 --no-cpu --no-roofline --no-f16 > gpurun_out/segbr_${br}_$rep.json 2> gpurun_out/segbr.err || { tail -20 gpurun_out/segbr.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/segbr_${br}_$rep.json'));print('seg x3 branches $br rep $rep', d['value'], d['device_images_per_s'])"
  done
done
bash tools/gpu_ctx_refine.sh n detect 8 3 x3 || exit 1
