#!/bin/bash
# In-context refinement of the committed yolo11s B=8 f16 table (tools/ctx_tune.py), then a bench A/B: committed
# table vs the refined one (copied over the committed path of this scratch tree).
cd "$(dirname "$0")/.." || exit 1
T=yolo-infer_amd/yolomi/tuned/s-detect-f16-b8-640x640.json
timeout -k 10 500 python -u tools/ctx_tune.py --model s --out gpurun_out/ctx_s.json > gpurun_out/ctx_s.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-roofline > gpurun_out/ctx_bench_base.json 2>/dev/null || exit 1
[ -f gpurun_out/ctx_s.json ] && cp gpurun_out/ctx_s.json $T
timeout -k 10 200 python bench.py --no-cpu --no-roofline > gpurun_out/ctx_bench_ref.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-roofline > gpurun_out/ctx_bench_ref2.json 2>/dev/null || exit 1
cp gpurun_out/ctx_s.json.bak $T 2>/dev/null
for f in base ref ref2; do python -c "import json; d=json.load(open('gpurun_out/ctx_bench_$f.json')); print('$f', d['value'], d['device_images_per_s'], d['config']['conv_tiles'])"; done
