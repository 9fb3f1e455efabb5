#!/bin/bash
# Round-5 fp8 datapath A/B: the fp8 plan's convs on the f16 MFMA over exactly widened e4m3 values (in-tree build)
# vs the fp8 MFMA (tools/ab/libF8N.so, the same sources built with -DYM_F8_NATIVE_MFMA): the fp8 GPU tests
# (layer-local exact-code rates, mAP against the fp8 oracle) under both, the int8 tests, then bench lines.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05h}
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
PYT="python -u -X faulthandler -m pytest -q -s -p no:cacheprovider --timeout 300 --timeout-method thread"
for step in ${STEPS:-f8 f8n quant bench}; do
  case $step in
    f8)  run f8tests 600 $PYT tests/test_gpu_fp8.py ;;
    f8n) YM_LIB=tools/ab/libF8N.so run f8tests_native 600 $PYT tests/test_gpu_fp8.py ;;
    quant) run quanttests 600 $PYT tests/test_gpu_quant.py ;;
    bench)
      for rep in 1 2; do
        for v in h n; do
          lib=yolo-infer_amd/yolomi/libyolomi.so
          [ $v = n ] && lib=tools/ab/libF8N.so
          YM_LIB=$lib run "bench_f8_${v}_$rep" 300 python -u bench.py --model n --dtype f8 --steps 50 --warmup 10 --no-cpu --no-roofline
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
