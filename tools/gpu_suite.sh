#!/bin/bash
# The whole GPU test suite (one process, its own limit) and the driver's smoke() on one box.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rs > gpurun_out/suite.log 2>&1; rc=$?
tail -8 gpurun_out/suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/suite.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/smoke.log
exit $rc
