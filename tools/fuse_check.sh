#!/bin/bash
# Fused conv pairs (GraphBuilder.fuse_pairs) on the GPU: parity tests, then per-op tables of yolo11n B=8 with the
# pairs fused (autotuned into gpurun_out/tune) and unfused (committed table), then the bench line.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp YM_TUNE_DIR="$PWD/gpurun_out/tune"
m=${1:-n}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gt.log 2>&1 || { tail -30 gpurun_out/gt.log; exit 1; }
tail -3 gpurun_out/gt.log
timeout -k 10 400 python tools/op_table.py --model $m > gpurun_out/optab_${m}_fused.txt 2>&1 || exit 1
YM_FUSE=0 timeout -k 10 300 python tools/op_table.py --model $m > gpurun_out/optab_${m}_unfused.txt 2>&1 || exit 1
tail -1 gpurun_out/optab_${m}_fused.txt gpurun_out/optab_${m}_unfused.txt
timeout -k 10 400 python bench.py --model $m > gpurun_out/bench_fused_$m.json 2> gpurun_out/bench_fused_$m.err || exit 1
cat gpurun_out/bench_fused_$m.json
for extra in "--model s" "--model s --task segment --batch 4"; do
  tag=$(echo $extra | tr -d ' -')
  timeout -k 10 400 python bench.py $extra > gpurun_out/bench_fused_$tag.json 2> gpurun_out/bench_fused_$tag.err || exit 1
  cat gpurun_out/bench_fused_$tag.json
done
