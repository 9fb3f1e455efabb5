#!/bin/bash
# bench.py at lanes 1/2/4 for yolo11n and yolo11s (no CPU baseline), one JSON line each under gpurun_out/
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
for m in n s; do for l in 1 2 4; do
  timeout -k 10 300 python bench.py --model $m --lanes $l --no-cpu > gpurun_out/lanes_${m}_${l}.json 2> gpurun_out/lanes_${m}_${l}.err
  rc=$?; echo "model $m lanes $l rc=$rc"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
