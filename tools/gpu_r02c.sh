#!/bin/bash
# Round-2 (third session) evidence on one GPU box: bench lines (s f16 default, n f16, s-seg B=4, n int8, n fp8, s f32 parity
# plan), a rocprofv3 --kernel-trace --stats run of the default bench command, separate FETCH_SIZE / WRITE_SIZE PMC
# passes for s and n and an SQ pass for s (per-op table).  Each GPU step has its own limit; a failing step ends it.
cd "$(dirname "$0")/.." || exit 1
D=gpurun_out/ev
mkdir -p $D
export TMPDIR=/tmp
R="$PWD"
step() { echo "[gpu_r02c] $1 $(date +%T)"; }
step bench_s;   timeout -k 10 400 python bench.py > $D/bench_s.json 2> $D/bench_s.err || exit 1
step bench_n;   timeout -k 10 400 python bench.py --model n > $D/bench_n.json 2> $D/bench_n.err || exit 1
step bench_seg; timeout -k 10 400 python bench.py --task segment --batch 4 > $D/bench_seg.json 2> $D/bench_seg.err || exit 1
step bench_i8;  timeout -k 10 500 python bench.py --model n --dtype i8 > $D/bench_n_i8.json 2> $D/bench_n_i8.err || exit 1
step bench_f8;  timeout -k 10 500 python bench.py --model n --dtype f8 > $D/bench_n_f8.json 2> $D/bench_n_f8.err || exit 1
step bench_f32; timeout -k 10 400 python bench.py --dtype f32 --steps 20 --warmup 3 --no-cpu > $D/bench_s_f32.json 2> $D/bench_s_f32.err || exit 1
step prof
rm -rf $D/prof_bench
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$D/prof_bench" -o run \
  -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/$D/prof_bench.log" 2>&1) || exit 1
for m in s n; do
  step pmc_$m
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$D/pmc_fetch_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m --ops-out "$R/$D/ops_$m.txt" > "$R/$D/pmc_fetch_$m.log" 2>&1) || exit 1
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$D/pmc_write_$m" -o run \
    -- python3 "$R/tools/pmc_forward.py" --model $m > "$R/$D/pmc_write_$m.log" 2>&1) || exit 1
done
step pmc_sq_s
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/$D/pmc_sq_s" -o run -- python3 "$R/tools/pmc_forward.py" --model s --reps 1 --ops-out "$R/$D/ops1_s.txt" > "$R/$D/pmc_sq_s.log" 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$D/pmc_fetch1_s" -o run \
  -- python3 "$R/tools/pmc_forward.py" --model s --reps 1 > "$R/$D/pmc_fetch1_s.log" 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$D/pmc_write1_s" -o run \
  -- python3 "$R/tools/pmc_forward.py" --model s --reps 1 > "$R/$D/pmc_write1_s.log" 2>&1) || exit 1
step done
