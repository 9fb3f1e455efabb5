#!/bin/bash
# Same-box A/B of the branch schedule (YM_BRANCHES: streams the op DAG is spread over; 1 = serial) on the x3 bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/br
for r in 1 2; do
  for b in 4 1 2 3; do
    YM_BRANCHES=$b timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-f16 --no-roofline \
      > gpurun_out/br/b${b}_$r.json 2> gpurun_out/br/b${b}_$r.err || exit 1
  done
done
