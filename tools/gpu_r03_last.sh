#!/bin/bash
# Last check at HEAD: the whole GPU suite, smoke(), the driver's default bench command, the segment bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/last
bash tools/gpu_suite.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/last/bench_s_x3.json 2> gpurun_out/last/bench_s_x3.err || { tail -20 gpurun_out/last/bench_s_x3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/last/bench_s_x3.json'));print('s x3', d['value'], d['device_images_per_s'], d['parity']['meets_tolerance'], d['roofline']['frac'], d['roofline'].get('frac_rocprof'), d['roofline'].get('mfma_busy'))"
timeout -k 10 400 python bench.py --task segment --batch 4 > gpurun_out/last/bench_seg_x3.json 2> gpurun_out/last/bench_seg_x3.err || { tail -20 gpurun_out/last/bench_seg_x3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/last/bench_seg_x3.json'));print('seg x3', d['value'], d['device_images_per_s'], d['parity']['meets_tolerance'])"
