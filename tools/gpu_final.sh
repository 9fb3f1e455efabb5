#!/bin/bash
# Round-end evidence on one GPU box: parity tests, bench lines (n f16 / s f16 / n i8 / s-seg f16), a rocprofv3
# --kernel-trace --stats run of the default bench command and separate FETCH_SIZE / WRITE_SIZE PMC passes for the
# n and s f16 workloads.  Every GPU step has its own time limit; a failing step ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
step() { echo "[gpu_final] $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
step bench_n
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
step bench_s
timeout -k 10 400 python bench.py --model s > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || exit 1
step bench_seg
timeout -k 10 400 python bench.py --model s --task segment --batch 4 > gpurun_out/bench_seg.json 2> gpurun_out/bench_seg.err || exit 1
step bench_i8
timeout -k 10 500 python bench.py --dtype i8 > gpurun_out/bench_i8.json 2> gpurun_out/bench_i8.err || exit 1
step prof
rm -rf gpurun_out/prof_bench
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o run \
  -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/prof_bench.log" 2>&1) || exit 1
for m in n s; do
  step pmc_$m
  rm -rf gpurun_out/pmc_fetch_$m gpurun_out/pmc_write_$m
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m > "$R/gpurun_out/pmc_fetch_$m.log" 2>&1) || exit 1
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m > "$R/gpurun_out/pmc_write_$m.log" 2>&1) || exit 1
done
step done
for f in bench bench_s bench_seg bench_i8; do python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', d['value'], d['device_images_per_s'], d['roofline']['frac'])"; done
