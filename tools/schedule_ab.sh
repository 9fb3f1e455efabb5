#!/bin/bash
# A/B of branch-stream count and lanes on the f16 detect benches (bench.py device and predict img/s).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab2
for m in s n; do
  for cfg in "YM_BRANCHES=4 L=1" "YM_BRANCHES=3 L=1" "YM_BRANCHES=2 L=1" "YM_BRANCHES=4 L=2"; do
    br=$(echo $cfg | sed 's/YM_BRANCHES=\([0-9]\).*/\1/'); l=$(echo $cfg | sed 's/.*L=//')
    YM_BRANCHES=$br timeout -k 10 200 python bench.py --model $m --no-cpu --no-roofline --steps 200 --lanes $l > gpurun_out/ab2/${m}_${br}_${l}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab2/${m}_${br}_${l}.json')); print('$m branches=$br lanes=$l', d['value'], d['device_images_per_s'])"
  done
done
