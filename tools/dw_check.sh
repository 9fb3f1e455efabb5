#!/bin/bash
# Depthwise kernel variants (YM_DW_PXT = pixels per thread: 4, 2, 1) on yolo11n/s B=8: parity tests, per-op tables.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
for m in n s; do for p in 4 2 1; do
  YM_DW_PXT=$p timeout -k 10 300 python tools/op_table.py --model $m > gpurun_out/optab_${m}_dw$p.txt 2>&1 || exit 1
  echo "$m pxt=$p: $(grep dwconv gpurun_out/optab_${m}_dw$p.txt | awk '{s+=$3} END {print s}') us dw; $(tail -1 gpurun_out/optab_${m}_dw$p.txt)"
done; done
