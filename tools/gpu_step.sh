#!/bin/bash
# Round-4 GPU session: x3 parity + multi-GPU receive path + kernel tests, smoke, bench, then the per-candidate conv
# timings of a fresh x3 yolo11s B=8 tune (YM_TUNE_LOG) with the per-op replay table.  Each step has its own limit;
# a GPU fault / abort / timeout ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run x3 700 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_dist.py tests/test_gpu_kernels.py -v -s --timeout 300 --timeout-method thread -k "not dwconv_variants"
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python -u bench.py --steps 20 --warmup 5
YM_TUNE_TABLES=0 YM_TUNE_LOG=1 YM_TUNE_DIR=gpurun_out/tune run optable 300 python -u tools/op_table.py --model s --dtype x3
# rocprof kernel trace of the headline bench command (timeline: tools/trace_timeline.py gpurun_out/prof 20 55)
R="$PWD"; export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline > "$R/gpurun_out/prof.log" 2>&1 )
echo "[prof] rc=$?" | tee -a gpurun_out/steps.log
# L2 warm-up A/B on the committed x3 table (same configs; YM_DMA_PF = largest M warmed: 12800 = 40x40 and 20x20 at B=8)
for pf in 0 12800; do
  YM_DMA_PF=$pf run optable_pf$pf 200 python -u tools/op_table.py --model s --dtype x3
  YM_DMA_PF=$pf run bench_pf$pf 300 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline
done
