#!/bin/bash
# x3 plan on the GPU: parity tests (tables tuned on this box land in gpurun_out/tune), per-op table, bench lines
# (serial and 4-stream branch schedule).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune" YM_PREFER_CACHE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 250 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -3 gpurun_out/x3_tests.log
timeout -k 10 200 python -u tools/op_table.py --model s --batch 8 --dtype x3 > gpurun_out/x3_s_b8_op_table.txt 2>&1 || { tail -20 gpurun_out/x3_s_b8_op_table.txt; exit 1; }
tail -1 gpurun_out/x3_s_b8_op_table.txt
for br in 1 4; do
  for m in s n; do
    YM_BRANCHES=$br timeout -k 10 300 python -u bench.py --model $m --steps 200 --no-cpu --no-f16 --no-roofline > gpurun_out/x3_bench_${m}_br$br.json 2> gpurun_out/x3_bench_${m}_br$br.err || { tail -20 gpurun_out/x3_bench_${m}_br$br.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/x3_bench_${m}_br$br.json'));print('$m br$br', d['value'], d['device_images_per_s'])"
  done
done
