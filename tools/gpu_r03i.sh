#!/bin/bash
# Round-3 lane-pair x3 epilogue stores: store-pattern probe, x3 + kernel GPU tests, x3 op tables (s / n B=8), the
# default bench line, then the whole GPU suite and smoke().
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/i
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/store_probe tools/store_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/store_probe > gpurun_out/i/store_probe.txt 2>&1 || { tail -5 gpurun_out/i/store_probe.txt; exit 1; }
grep -E "pair" gpurun_out/i/store_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/i/x3_tests.log 2>&1 || { tail -40 gpurun_out/i/x3_tests.log; exit 1; }
tail -2 gpurun_out/i/x3_tests.log
for m in s n; do
  timeout -k 10 300 python -u tools/op_table.py --model $m --dtype x3 > gpurun_out/i/op_table_${m}_x3.txt 2>&1 || { tail -20 gpurun_out/i/op_table_${m}_x3.txt; exit 1; }
  tail -1 gpurun_out/i/op_table_${m}_x3.txt
done
timeout -k 10 400 python bench.py > gpurun_out/i/bench_s_x3.json 2> gpurun_out/i/bench_s_x3.err || { tail -20 gpurun_out/i/bench_s_x3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/i/bench_s_x3.json'));print('s x3', d['value'], d['device_images_per_s'], d['parity']['meets_tolerance'], d['roofline']['frac'])"
bash tools/gpu_suite.sh
