#!/bin/bash
# Round-2 evidence on one GPU box: bench lines (s f16 default, n f16, s f32 parity plan, s-seg B=4, n int8), a
# rocprofv3 --kernel-trace --stats run of the default bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes for
# s and n, and an SQ pass (MFMA busy, wave waits, GRBM) for s -> per-op table.  Each GPU step has its own limit; a
# failing step ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
step() { echo "[gpu_r02] $1 $(date +%T)"; }
SKIP_BENCH=${SKIP_BENCH:-0}
if [ "$SKIP_BENCH" = 0 ]; then
step bench_s
timeout -k 10 400 python bench.py > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || exit 1
step bench_n
timeout -k 10 400 python bench.py --model n > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || exit 1
step bench_s_f32
timeout -k 10 400 python bench.py --dtype f32 --steps 20 --warmup 3 > gpurun_out/bench_s_f32.json 2> gpurun_out/bench_s_f32.err || exit 1
step bench_seg
timeout -k 10 400 python bench.py --task segment --batch 4 > gpurun_out/bench_seg.json 2> gpurun_out/bench_seg.err || exit 1
step bench_i8
timeout -k 10 500 python bench.py --model n --dtype i8 > gpurun_out/bench_n_i8.json 2> gpurun_out/bench_n_i8.err || exit 1
fi
step prof
rm -rf gpurun_out/prof_bench
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" -o run \
  -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/prof_bench.log" 2>&1) || exit 1
for m in s n; do
  step pmc_$m
  rm -rf gpurun_out/pmc_fetch_$m gpurun_out/pmc_write_$m
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m --ops-out "$R/gpurun_out/ops_$m.txt" > "$R/gpurun_out/pmc_fetch_$m.log" 2>&1) || exit 1
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m > "$R/gpurun_out/pmc_write_$m.log" 2>&1) || exit 1
done
step pmc_sq_s
rm -rf gpurun_out/pmc_sq_s
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/gpurun_out/pmc_sq_s" -o run -- python3 "$R/tools/pmc_forward.py" --model s > "$R/gpurun_out/pmc_sq_s.log" 2>&1) || exit 1
step done
