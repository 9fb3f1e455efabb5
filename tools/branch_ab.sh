#!/bin/bash
# A/B of the branch schedule (YM_BRANCHES=1 serial vs the default 4 streams) on every bench workload: one bench.py
# line per (workload, schedule), device img/s printed.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
for w in "--model s" "--model n" "--task segment --batch 4" "--model n --dtype i8" "--model n --dtype f8"; do
  for br in 1 4; do
    tag=$(echo "$w b$br" | tr ' -' '__')
    YM_BRANCHES=$br timeout -k 10 300 python bench.py $w --no-cpu --no-roofline --steps 100 > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/$tag.json')); print('$w', 'branches=$br', d['value'], d['device_images_per_s'])"
  done
done
