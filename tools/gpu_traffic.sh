#!/bin/bash
# Bench (s, n) + FETCH_SIZE / WRITE_SIZE passes for the s forward -> per-op traffic table (gpurun_out/ops_tab.md).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
M=${1:-s}
timeout -k 10 300 python bench.py --model $M --no-cpu > gpurun_out/bench_$M.json 2> gpurun_out/bench_$M.err || exit 1
rm -rf gpurun_out/pmc_fetch_$M gpurun_out/pmc_write_$M
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch_$M" -o run \
  -- python3 "$R/tools/pmc_forward.py" --model $M --ops-out "$R/gpurun_out/ops_$M.txt" > "$R/gpurun_out/pmc_fetch_$M.log" 2>&1) || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write_$M" -o run \
  -- python3 "$R/tools/pmc_forward.py" --model $M > "$R/gpurun_out/pmc_write_$M.log" 2>&1) || exit 1
