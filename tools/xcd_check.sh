#!/bin/bash
# XCD-contiguous tile order: GPU parity tests (incl. int8), then per-op tables of yolo11n/s B=8 on the committed
# conv tables (compare with the previous order's tables), then the bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp YM_TUNE_DIR="$PWD/gpurun_out/tune_xcd"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
for m in n s; do
  timeout -k 10 300 python tools/op_table.py --model $m > gpurun_out/optab_${m}_xcd.txt 2>&1 || exit 1
  tail -1 gpurun_out/optab_${m}_xcd.txt
done
timeout -k 10 300 python tools/op_table.py --model n --dtype i8 > gpurun_out/optab_n_i8_xcd.txt 2>&1 || exit 1
tail -1 gpurun_out/optab_n_i8_xcd.txt
