#!/bin/bash
# Segment predict path (mask slot cap 1.25x): the mask / segment GPU tests, two bench lines, a rocprof kernel trace.
cd "$(dirname "$0")/.." || exit 1
R="$PWD"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "segment or mask or seg" --timeout 200 --timeout-method thread > gpurun_out/seg_tests.log 2>&1 || { tail -30 gpurun_out/seg_tests.log; exit 1; }
tail -2 gpurun_out/seg_tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --task segment --batch 4 --no-cpu --no-roofline --no-f16 > gpurun_out/seg_bench_$r.json 2> gpurun_out/seg_bench.err || { tail -20 gpurun_out/seg_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/seg_bench_$r.json'));print('seg x3', d['value'], d['device_images_per_s'], round(d['value']/d['device_images_per_s'],3))"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/segprof" -o run -- python3 "$R/bench.py" --task segment --batch 4 --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline > "$R/gpurun_out/segprof.log" 2>&1 || { tail -5 "$R/gpurun_out/segprof.log"; exit 1; }
