#!/bin/bash
# Round-5 second box: first-call predict() diagnostic, the x3 parity tests, then a same-box A/B of the conv_dma
# kernarg warm-up (in-tree build vs tools/ab/libA.so built with -DYM_NO_WARM): per-op replay tables and bench lines.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05b}
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
for step in ${STEPS:-calls x3tests ab}; do
  case $step in
    calls) run calls 300 python -u tools/predict_calls_check.py s 8 ;;
    x3tests) run x3tests 900 python -u -X faulthandler -m pytest tests/test_gpu_x3.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab)  # variants: w = in-tree (kernarg warm-up in conv_dma), nw = tools/ab/libA.so (built with -DYM_NO_WARM);
         # each twice, interleaved
      for rep in 1 2; do
        for v in w nw; do
          lib=yolo-infer_amd/yolomi/libyolomi.so
          [ $v = nw ] && lib=tools/ab/libA.so
          YM_LIB=$lib run "optable_${v}_$rep" 200 python -u tools/op_table.py --model s --dtype x3
          YM_LIB=$lib run "bench_${v}_$rep" 300 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
