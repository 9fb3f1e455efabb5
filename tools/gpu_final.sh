#!/bin/bash
# Round-end evidence on one box: smoke, the whole GPU suite, the bench lines (headline yolo11s x3, yolo11n x3,
# yolo11s-seg, the yolo11n PTQ int8 / fp8 lines and f16 beside them), the per-op replay table, rocprofv3 stats and
# PMC passes of the headline bench command, and the per-op SQ table (MFMA busy) of one headline forward (sq).  Each GPU step under its own limit; a fatal status ends it.
#   TAG=r05z STEPS="smoke suite" bash tools/gpu_final.sh        (default: every step; output gpurun_out/$TAG)
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-final}
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
for step in ${STEPS:-smoke suite bench_s bench_n bench_seg bench_ptq optable prof pmc}; do
  case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    suite) run suite 1100 python -u -X faulthandler -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench_s) run bench_s 400 python -u bench.py ;;
    bench_n) run bench_n 400 python -u bench.py --model n --no-f16 ;;
    bench_seg) run bench_seg 400 python -u bench.py --task segment --batch 4 --no-f16 ;;
    bench_ptq) run bench_n_i8 400 python -u bench.py --model n --dtype i8
               run bench_n_f8 400 python -u bench.py --model n --dtype f8
               run bench_n_f16 400 python -u bench.py --model n --dtype f16 --no-cpu ;;
    optable) run optable 200 python -u tools/op_table.py --model s --dtype x3 ;;
    files) run files 900 python -u -X faulthandler -m pytest $TEST_FILES -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ktests) run ktests 400 python -u -X faulthandler -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 200 --timeout-method thread ${KTESTS_K:+-k "$KTESTS_K"} ;;
    ab) for v in 0 1 0 1; do  # same-box A/B of an environment switch AB_VAR (e.g. YM_CHAIN, YM_STEMFUSE)
          export "$AB_VAR=$v"
          run "ab_${AB_VAR}_$v" 300 python -u bench.py --no-cpu --no-f16 --no-roofline --steps 400
          mv "$OUT/ab_${AB_VAR}_$v.log" "$OUT/ab_${AB_VAR}_${v}_$((++n))"; done
        export "$AB_VAR=1"
        (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$GRAFT_REPO_ROOT/$OUT/prof_ab" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 \
          --warmup 10 --no-cpu --no-f16 --no-roofline > "$GRAFT_REPO_ROOT/$OUT/prof_ab.log" 2>&1); rc=$?
        unset "$AB_VAR"
        echo "[prof_ab] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
        if [ $rc -ne 0 ]; then exit $rc; fi ;;
    sq) bash tools/gpu_sq_table.sh "${TAG:-final}" --model s --dtype x3 > "$OUT/sq.log" 2>&1; rc=$?
        echo "[sq] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
        if [ $rc -ne 0 ]; then exit $rc; fi ;;
    conf) run conf_timing 300 python -u tools/conf_timing.py s 8 ;;
    profconf) (cd /tmp && CONFS=0.001 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/$OUT/prof_conf" -o run -- python3 "$GRAFT_REPO_ROOT/tools/conf_timing.py" s 8 \
             > "$GRAFT_REPO_ROOT/$OUT/prof_conf.log" 2>&1); rc=$?
          echo "[profconf] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
          if [ $rc -ne 0 ]; then exit $rc; fi ;;
    prof) (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 \
             --warmup 10 --no-cpu --no-f16 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.log" 2>&1); rc=$?
          echo "[prof] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
          if [ $rc -ne 0 ]; then exit $rc; fi
          python3 tools/trace_timeline.py "$OUT/prof" 20 55 > "$OUT/timeline.txt" 2>&1 ;;
    pmc) (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$GRAFT_REPO_ROOT/$OUT/pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pmc_forward.py" --model s --dtype x3 \
             > "$GRAFT_REPO_ROOT/$OUT/pmc_fetch.log" 2>&1); rc=$?
         echo "[pmc_fetch] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
         if [ $rc -ne 0 ]; then exit $rc; fi
         (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$GRAFT_REPO_ROOT/$OUT/pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pmc_forward.py" --model s --dtype x3 \
             > "$GRAFT_REPO_ROOT/$OUT/pmc_write.log" 2>&1); rc=$?
         echo "[pmc_write] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
         if [ $rc -ne 0 ]; then exit $rc; fi ;;
  esac
done
echo done >> "$OUT/steps.log"
