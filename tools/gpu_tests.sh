#!/bin/bash
# The whole GPU test suite on one box (one process, its own limit).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs "$@" > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -6 gpurun_out/gpu_tests.log
