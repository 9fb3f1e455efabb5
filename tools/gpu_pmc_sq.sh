#!/bin/bash
# Two SQ counter passes + one TCC pass over eager forwards of the bench workload; per-op table into gpurun_out/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
ARGS="$*"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
  --output-format csv -d "$R/gpurun_out/pmc_sq1" -o run -- python3 "$R/tools/pmc_forward.py" --reps 1 --ops-out "$R/gpurun_out/ops.txt" $ARGS > "$R/gpurun_out/pmc_sq1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/gpurun_out/pmc_sq2" -o run -- python3 "$R/tools/pmc_forward.py" --reps 1 $ARGS > "$R/gpurun_out/pmc_sq2.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum \
  --output-format csv -d "$R/gpurun_out/pmc_tcc" -o run -- python3 "$R/tools/pmc_forward.py" --reps 1 $ARGS > "$R/gpurun_out/pmc_tcc.log" 2>&1 || exit $?
cd "$R" && python3 tools/pmc_ops.py gpurun_out/ops.txt gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 gpurun_out/pmc_tcc > gpurun_out/pmc_ops.txt
