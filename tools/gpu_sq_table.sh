#!/bin/bash
# Per-op PMC table of one eager forward: FETCH_SIZE, WRITE_SIZE and one SQ pass (MFMA busy, wave waits, GRBM), each
# its own rocprofv3 run under its own time limit; then (locally, after the merge) tools/op_pmc_table.py.
#   bash tools/gpu_sq_table.sh <tag> [pmc_forward.py args]
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
TAG=$1; shift
ARGS="$*"
D="$R/gpurun_out/sq_$TAG"
rm -rf "$D"; mkdir -p "$D"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run \
  -- python3 "$R/tools/pmc_forward.py" --reps 1 --ops-out "$D/ops.txt" $ARGS > "$D/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/write" -o run \
  -- python3 "$R/tools/pmc_forward.py" --reps 1 $ARGS > "$D/write.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d "$D/sq" -o run -- python3 "$R/tools/pmc_forward.py" --reps 1 $ARGS > "$D/sq.log" 2>&1 || exit $?
