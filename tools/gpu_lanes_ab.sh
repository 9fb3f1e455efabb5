#!/bin/bash
# A/B of the x3 plan's lanes (concurrent batch slices per forward graph) and branch streams, yolo11s B=8, interleaved.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
for rep in 1 2; do
  for cfg in "1 4" "2 4" "1 2" "2 2"; do
    set -- $cfg
    YM_BRANCHES=$2 timeout -k 10 200 python bench.py --dtype x3 --lanes $1 --no-cpu --no-roofline --no-f16 > gpurun_out/lanes_$1_$2_$rep.json 2> gpurun_out/lanes.err || { tail -20 gpurun_out/lanes.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lanes_$1_$2_$rep.json'));print('lanes $1 branches $2 rep $rep', d['value'], d['device_images_per_s'])"
  done
done
