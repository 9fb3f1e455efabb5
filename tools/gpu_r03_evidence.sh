#!/bin/bash
# Round-3 evidence at HEAD for the benched x3 plan (yolo11s B=8): bench line, rocprofv3 kernel stats of the same bench
# command (x3 only), FETCH/WRITE PMC passes of tools/pmc_forward.py, and the per-op SQ table passes.  Every GPU step
# has its own limit; a fault / abort / timeout stops the script.  Summaries are built locally afterwards:
#   python tools/rocprof_summary.py stats gpurun_out/ev3/prof <tag> "<workload>"
#   python tools/rocprof_summary.py pmc gpurun_out/ev3/pmc_fetch gpurun_out/ev3/pmc_write <tag> "<workload>"
#   YM_OPS_WORKLOAD="<workload>" python tools/op_pmc_table.py gpurun_out/sq_<tag>/ops.txt <tag> gpurun_out/sq_<tag>/{fetch,write,sq}
cd "$(dirname "$0")/.." || exit 1
R="$PWD"
mkdir -p gpurun_out/ev3
export TMPDIR=/tmp
MODEL=${MODEL:-s}; DT=${DT:-x3}; TAG=${TAG:-r03c_s_b8_x3}
step() { echo "[ev3] $1 $(date +%T)"; }
step bench
timeout -k 10 400 python bench.py --model $MODEL --dtype $DT > gpurun_out/ev3/bench.json 2> gpurun_out/ev3/bench.err || { tail -20 gpurun_out/ev3/bench.err; exit 1; }
cat gpurun_out/ev3/bench.json
step prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ev3/prof" -o run -- \
  python3 "$R/bench.py" --model $MODEL --dtype $DT --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline > "$R/gpurun_out/ev3/prof.log" 2>&1 || { tail -20 "$R/gpurun_out/ev3/prof.log"; exit 1; }
step pmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/ev3/pmc_fetch" -o run -- \
  python3 "$R/tools/pmc_forward.py" --model $MODEL --dtype $DT > "$R/gpurun_out/ev3/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/ev3/pmc_write" -o run -- \
  python3 "$R/tools/pmc_forward.py" --model $MODEL --dtype $DT > "$R/gpurun_out/ev3/pmc_write.log" 2>&1 || exit $?
cd "$R"
step sq
bash tools/gpu_sq_table.sh $TAG --model $MODEL --dtype $DT || exit $?
step done
