#!/bin/bash
# Round-5 NMS IoU early-out (no intersection: no division) on top of the blocked path (tools/ab/libBlk.so), same tests
# vs confidence threshold and the headline bench, new build vs the previous one (tools/ab/libBlk.so), interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05t}
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
    tests) run nmstests 900 $PYT tests/test_gpu_parity.py tests/test_gpu_x3.py -k "nms or max_nms or low_conf or 1280 or kwargs or sizes or non_square" ;;
    ab)
      for rep in 1 2; do
        for v in new prev; do
          lib=yolo-infer_amd/yolomi/libyolomi.so
          [ $v = prev ] && lib=tools/ab/libBlk.so
          YM_LIB=$lib run "conf_${v}_$rep" 300 python -u tools/conf_timing.py s 8
          YM_LIB=$lib run "bench_${v}_$rep" 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
