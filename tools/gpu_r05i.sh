#!/bin/bash
# Round-5 depthwise -> 1x1 K split (csrc/ym_conv_dwpw.hip SPLIT): the fused-kernel tests, a table for the plan with the
# P4 / P5 depthwise ops fused too (tools/retable.py under YM_DW_FUSE_STRIDES=8,16,32), then a same-box A/B against
# the committed plan (P3 only): per-op replay tables and bench lines, interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05i}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/steps.log"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
PYT="python -u -X faulthandler -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for step in ${STEPS:-test retable ab}; do
  case $step in
    test) run dwpw_tests 600 $PYT tests/test_gpu_kernels.py -k fused_depthwise ;;
    retable) YM_DW_FUSE_STRIDES=8,16,32 YM_TUNE_LOG=1 run retable 600 python -u tools/retable.py s:detect:x3:8 ;;
    ab)
      mkdir -p "$OUT/tune" && cp gpurun_out/tuned/s-detect-x3-b8-640x640.json "$OUT/tune/" || exit 1
      for rep in 1 2; do
        for v in p3 all; do
          st=""; [ $v = all ] && st=8,16,32
          YM_DW_FUSE_STRIDES=$st YM_TUNE_DIR=$OUT/tune YM_PREFER_CACHE=1 run "optable_${v}_$rep" 200 python -u tools/op_table.py --model s --dtype x3
          YM_DW_FUSE_STRIDES=$st YM_TUNE_DIR=$OUT/tune YM_PREFER_CACHE=1 run "bench_${v}_$rep" 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
