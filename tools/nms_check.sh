#!/bin/bash
# NMS kernel: GPU parity tests, then rocprofv3 kernel trace of tools/nms_probe.py (20 eager forwards per conf).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -1 gpurun_out/gt.log
rm -rf gpurun_out/nmsp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/nmsp" -o run \
  -- python3 "$R/tools/nms_probe.py" > "$R/gpurun_out/nmsp.log" 2>&1) || exit 1
grep conf gpurun_out/nmsp.log
python3 tools/nms_summary.py gpurun_out/nmsp
