#!/bin/bash
# Round-5 first box: smoke, the whole GPU suite (no -x: every failure listed), the headline bench line, the
# float64 bisect of the x3 plan's coordinate error, and per-op replay tables of the f32 and x3 plans (the exact-f32
# MFMA vs x3 A/B on the 20x20 layers).  Each GPU step under its own limit; a fatal status ends the script.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05a}
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
for step in ${STEPS:-smoke suite bench bisect optable_f32 optable_x3}; do
  case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    suite) run suite 1200 python -u -X faulthandler -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run bench 400 python -u bench.py --steps 20 --warmup 5 ;;
    bisect) run bisect 400 python -u tools/x3_bisect.py s 8 ;;
    optable_f32) run optable_f32 300 python -u tools/op_table.py --model s --dtype f32 ;;
    optable_x3) run optable_x3 200 python -u tools/op_table.py --model s --dtype x3 ;;
  esac
done
echo done >> "$OUT/steps.log"
