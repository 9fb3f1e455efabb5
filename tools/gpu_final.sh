#!/bin/bash
# Round-end evidence on one box: smoke, the whole GPU suite, the three bench lines, rocprofv3 stats + PMC passes of
# the headline bench command, and the per-op replay table.  Each GPU step under its own limit; a fatal status ends it.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/final
export TMPDIR=/tmp
: > gpurun_out/final/steps.log
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/final/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" | tee -a gpurun_out/final/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run suite 1200 python -u -X faulthandler -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bench_s 400 python -u bench.py
run bench_n 400 python -u bench.py --model n --no-f16
run bench_seg 400 python -u bench.py --task segment --batch 4 --no-f16
run optable 200 python -u tools/op_table.py --model s --dtype x3
bash tools/gpu_round.sh prof > gpurun_out/final/prof_step.log 2>&1 || exit 1
PMC_ARGS="--model s --dtype x3" bash tools/gpu_round.sh pmc > gpurun_out/final/pmc_step.log 2>&1 || exit 1
echo done >> gpurun_out/final/steps.log
