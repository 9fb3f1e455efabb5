#!/bin/bash
# Round-5 evidence box: smoke, the whole GPU suite, the headline bench line, the x3 op table, the float64 bisect, and a
# rocprofv3 kernel-trace/stats run of the bench command (timeline: tools/trace_timeline.py).  Each GPU step under its
# own limit; a fatal status ends the script.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05c}
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
for step in ${STEPS:-smoke suite bench optable bisect prof}; do
  case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    suite) run suite 1200 python -u -X faulthandler -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    x3tests) run x3tests 900 python -u -X faulthandler -m pytest tests/test_gpu_x3.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run bench 400 python -u bench.py --steps 20 --warmup 5 ;;
    optable) run optable 200 python -u tools/op_table.py --model s --dtype x3 ;;
    bisect) run bisect 400 python -u tools/x3_bisect.py s 8 ;;
    prof) (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 \
             --warmup 10 --no-cpu --no-f16 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.log" 2>&1); rc=$?
          echo "[prof] rc=$rc $(date +%T)" | tee -a "$OUT/steps.log"
          if [ $rc -ne 0 ]; then exit $rc; fi
          python3 tools/trace_timeline.py "$OUT/prof" 20 55 > "$OUT/timeline.txt" 2>&1 ;;
  esac
done
echo done >> "$OUT/steps.log"
