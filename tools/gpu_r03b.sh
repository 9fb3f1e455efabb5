#!/bin/bash
# Round-3 x3 iteration: x3 + kernel-variant GPU tests (tables tuned on this box land in gpurun_out/tune), per-op
# replay tables of yolo11s / yolo11n x3 B=8, and a bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -3 gpurun_out/x3_tests.log
for m in s n; do
  timeout -k 10 300 python -u tools/op_table.py --model $m --dtype x3 > gpurun_out/op_table_${m}_x3.txt 2>&1 || { tail -20 gpurun_out/op_table_${m}_x3.txt; exit 1; }
  tail -1 gpurun_out/op_table_${m}_x3.txt
done
timeout -k 10 300 python -u bench.py --no-cpu --no-roofline > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err || { tail -20 gpurun_out/bench_x3.err; exit 1; }
cat gpurun_out/bench_x3.json
