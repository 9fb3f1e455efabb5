#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 bash tools/gpu_probe.sh; echo "[probe] rc=$?"
