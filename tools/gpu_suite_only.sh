#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/final
timeout -k 10 1200 python -u -X faulthandler -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final/suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/final/suite.log
