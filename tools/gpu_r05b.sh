#!/bin/bash
# Round-5 A/B of the staggered wave groups of the x3 LDS-DMA kernels (conv_dma STG, YM_DMA_STG): x3 parity tests
# with the stagger on (the default), then per-op replay tables and quick bench lines with it off / on, same box.
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
for step in ${STEPS:-x3tests ab}; do
  case $step in
    x3tests) run x3tests 900 python -u -X faulthandler -m pytest tests/test_gpu_x3.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab)  # variants: s1 = in-tree (staggered groups + kernarg warm-up), s0 = in-tree with YM_DMA_STG=0, nw = tools/ab/libA.so
         # (staggered, no warm-up); each twice, interleaved
      for rep in 1 2; do
        for v in s1 s0 nw; do
          lib=yolo-infer_amd/yolomi/libyolomi.so; stg=1
          [ $v = s0 ] && stg=0
          [ $v = nw ] && lib=tools/ab/libA.so
          YM_LIB=$lib YM_DMA_STG=$stg run "optable_${v}_$rep" 200 python -u tools/op_table.py --model s --dtype x3
          YM_LIB=$lib YM_DMA_STG=$stg run "bench_${v}_$rep" 300 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
