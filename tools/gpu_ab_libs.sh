#!/bin/bash
# Same-box A/B of library builds (YM_LIB): the op table and the bench of yolo11s x3 B=8 with each variant.
#   tools/ab/libA.so, tools/ab/libC.so (built on the CPU side), and the in-tree build as B
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
: > gpurun_out/ab/steps.log
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/ab/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/ab/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
export YM_FUSE_DW=${YM_FUSE_DW:-0}
for v in A B C A B C; do
  lib=tools/ab/lib$v.so; [ $v = B ] && lib=yolo-infer_amd/yolomi/libyolomi.so
  YM_LIB=$lib run "optable_$v" 200 python -u tools/op_table.py --model s --dtype x3
  mv "gpurun_out/ab/optable_$v.log" "gpurun_out/ab/optable_${v}_$((++n)).log"
done
for v in A B C; do
  lib=tools/ab/lib$v.so; [ $v = B ] && lib=yolo-infer_amd/yolomi/libyolomi.so
  YM_LIB=$lib run "bench_$v" 300 python -u bench.py --steps 50 --warmup 10 --no-cpu --no-f16
done
