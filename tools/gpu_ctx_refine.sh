#!/bin/bash
# In-context refinement of a committed f16 B=8 detect table (tools/ctx_tune.py; $1 = model scale, default s), then a
# bench A/B: committed table vs the refined one (copied over the committed path of this scratch tree).
cd "$(dirname "$0")/.." || exit 1
M=${1:-s}
T=yolo-infer_amd/yolomi/tuned/$M-detect-f16-b8-640x640.json
timeout -k 10 500 python -u tools/ctx_tune.py --model $M --out gpurun_out/ctx_$M.json > gpurun_out/ctx_$M.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model $M --no-cpu --no-roofline > gpurun_out/ctx_bench_${M}_base.json 2>/dev/null || exit 1
[ -f gpurun_out/ctx_$M.json ] && cp gpurun_out/ctx_$M.json $T
for f in ref ref2; do
  timeout -k 10 200 python bench.py --model $M --no-cpu --no-roofline > gpurun_out/ctx_bench_${M}_$f.json 2>/dev/null || exit 1
done
for f in base ref ref2; do python -c "import json; d=json.load(open('gpurun_out/ctx_bench_${M}_$f.json')); print('$M $f', d['value'], d['device_images_per_s'], d['config']['conv_tiles'])"; done
