#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/steps.log
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run fpairs 700 python -u -m pytest tests/test_gpu_x3.py -q -x --timeout 600 --timeout-method thread -k "fused_pairs"
rm -rf gpurun_out/tuned
YM_RETABLE_OPS=model.1+cv1,model.3+cv1,model.5+cv1,model.23.cv2.0.1+2,model.23.cv2.1.1+2,model.23.cv2.2.1+2,model.23.proto.cv2+cv3,model.23.cv4.0.1+2,model.23.cv4.1.1+2,model.23.cv4.2.1+2 run retable 400 python -u tools/retable.py
cp gpurun_out/tuned/*.json yolo-infer_amd/yolomi/tuned/ 2>/dev/null
run optable 200 python -u tools/op_table.py --model s --dtype x3
run bench 400 python -u bench.py --steps 100 --warmup 10 --no-cpu
