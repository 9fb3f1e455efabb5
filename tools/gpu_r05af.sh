#!/bin/bash
# Round-5 conv_dma tile-map divisions set on the host (multiply-shift divisors), vs the previous
# build (tools/ab/libPrev.so): x3 + kernel tests on the new build, then per-op replay tables and bench lines, interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05af}
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
for step in ${STEPS:-tests ab}; do
  case $step in
    tests) run x3tests 900 $PYT tests/test_gpu_x3.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "x3 or dma or halo or fused or bneck or split" ;;
    ab)
      for rep in 1 2; do
        for v in new prev; do
          lib=yolo-infer_amd/yolomi/libyolomi.so
          [ $v = prev ] && lib=tools/ab/libPrev.so
          YM_LIB=$lib run "optable_${v}_$rep" 200 python -u tools/op_table.py --model s --dtype x3
          YM_LIB=$lib run "bench_${v}_$rep" 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
