#!/bin/bash
# GPU session: x3 parity tests (float64-slack bar), smoke, bench, DMA cycle-stamp probes.  Each step has its own
# limit; a GPU fault / abort / timeout ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/steps.log
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run x3 600 python -u -m pytest tests/test_gpu_x3.py -v -s --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python -u bench.py --steps 20 --warmup 5
run probe 300 bash tools/gpu_probe.sh
