#!/bin/bash
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
run tests 900 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread
: > gpurun_out/nms_phases.log
for d in 0 1 6; do
  YM_NMS_DBG=$d timeout -k 10 120 python -u tools/nms_phases.py >> gpurun_out/nms_phases.log 2>&1 || { echo "nms rc=$?" >> gpurun_out/steps.log; exit 1; }
done
run bench 400 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-f16
