#!/bin/bash
# Re-tune the f16 tables of the given workloads (tools/gpu_tune.sh), then bench yolo11s / yolo11n B=8 on them.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_tune.sh "$@" || exit 1
export YM_TUNE_DIR="$PWD/gpurun_out/tune"
for m in s n; do
  echo "[bench] $m $(date +%T)"
  timeout -k 10 300 python bench.py --model $m --no-cpu > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || exit 1
  cat gpurun_out/bench_$m.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['device_images_per_s'], d['roofline']['frac'], d['roofline'].get('per_launch_roofline_frac'))"
done
