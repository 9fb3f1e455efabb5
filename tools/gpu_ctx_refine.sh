#!/bin/bash
# In-context refinement of a committed table (tools/ctx_tune.py; $1 = scale (s), $2 = task (detect), $3 = batch
# (8), $4 = candidates per op (3), $5 = plan dtype (f16)), then a bench A/B: committed table vs the refined one (copied
# over the committed path of this scratch tree).
cd "$(dirname "$0")/.." || exit 1
M=${1:-s}; TK=${2:-detect}; B=${3:-8}; DT=${5:-f16}
T=yolo-infer_amd/yolomi/tuned/$M-$TK-$DT-b$B-640x640.json
O=gpurun_out/ctx_${M}_${TK}_$DT.json
timeout -k 10 500 python -u tools/ctx_tune.py --model $M --task $TK --batch $B --dtype $DT --top ${4:-3} --out $O > gpurun_out/ctx_${M}_${TK}_$DT.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model $M --task $TK --batch $B --dtype $DT --no-f16 --no-cpu --no-roofline > gpurun_out/ctx_bench_${M}_${TK}_base.json 2>/dev/null || exit 1
[ -f $O ] && cp $O $T
for f in ref ref2; do
  timeout -k 10 200 python bench.py --model $M --task $TK --batch $B --dtype $DT --no-f16 --no-cpu --no-roofline > gpurun_out/ctx_bench_${M}_${TK}_$f.json 2>/dev/null || exit 1
done
for f in base ref ref2; do python -c "import json; d=json.load(open('gpurun_out/ctx_bench_${M}_${TK}_$f.json')); print('$M $TK $f', d['value'], d['device_images_per_s'], d['config']['conv_tiles'])"; done
