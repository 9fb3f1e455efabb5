#!/bin/bash
# Same-box A/B of the branch-stream placement rule (YM_SCHED: default = the latest dependency in program order,
# crit = the dependency expected to finish last) on the x3 bench, plus the schedule-invariance tests under crit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/sched
YM_SCHED=crit timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread \
  -k "branch_schedule or graph_replay" > gpurun_out/sched/tests.log 2>&1 || exit 1
for r in 1 2; do
  for m in def crit; do
    YM_SCHED=$m timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-f16 --no-roofline \
      > gpurun_out/sched/${m}_$r.json 2>/dev/null || exit 1
  done
done
