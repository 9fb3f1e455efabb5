#!/bin/bash
# Round-5 NMS sorts inlined (a called sort took generic-pointer flat accesses to LDS and spilled SGPRs), vs the called one: NMS tests,
# the kernel's time at conf 0.001 under rocprofv3 (whole kernel, and YM_NMS_DBG=10: the blocked path's sort alone),
# then forward time vs conf, new build vs tools/ab/libSort.so.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05z}
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
for step in ${STEPS:-tests prof ab}; do
  case $step in
    tests) run nmstests 900 $PYT tests/test_gpu_parity.py tests/test_gpu_x3.py -k "nms or max_nms or low_conf or 1280 or kwargs or sizes or non_square" ;;
    prof) for d in 0 10 11; do
            (cd /tmp && YM_NMS_DBG=$d CONFS=0.001 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
               -d "$GRAFT_REPO_ROOT/$OUT/prof_$d" -o run -- python3 "$GRAFT_REPO_ROOT/tools/conf_timing.py" s 8 \
               > "$GRAFT_REPO_ROOT/$OUT/prof_$d.log" 2>&1); rc=$?
            echo "[prof_$d] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
            if [ $rc -ne 0 ]; then exit $rc; fi
          done ;;
    ab)
      for rep in 1 2; do
        for v in new prev; do
          lib=yolo-infer_amd/yolomi/libyolomi.so
          [ $v = prev ] && lib=tools/ab/libSort.so
          YM_LIB=$lib run "conf_${v}_$rep" 300 python -u tools/conf_timing.py s 8
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
