#!/bin/bash
# x3 plan on the GPU: parity tests (tables tuned on this box land in gpurun_out/tune), per-op table, bench lines.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tune
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -x -v --timeout 200 --timeout-method thread > gpurun_out/x3_tests.log 2>&1 || { tail -40 gpurun_out/x3_tests.log; exit 1; }
tail -3 gpurun_out/x3_tests.log
timeout -k 10 200 python -u tools/op_table.py --model s --batch 8 --dtype x3 > gpurun_out/x3_s_b8_op_table.txt 2>&1 || { tail -20 gpurun_out/x3_s_b8_op_table.txt; exit 1; }
tail -3 gpurun_out/x3_s_b8_op_table.txt
for m in s n; do
  timeout -k 10 300 python -u bench.py --dtype x3 --model $m --steps 100 --no-cpu > gpurun_out/x3_bench_$m.json 2> gpurun_out/x3_bench_$m.err || { tail -20 gpurun_out/x3_bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/x3_bench_$m.json'));print('$m', d['value'], d['device_images_per_s'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
done
