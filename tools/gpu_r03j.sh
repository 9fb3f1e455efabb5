#!/bin/bash
# Round-3 evidence after the lane-pair x3 epilogue stores (x3 plans only; the f16 / int8 / fp8 / f32 kernels are
# unchanged): bench lines of the x3 BASELINE configs, rocprofv3 kernel stats of the headline bench command,
# FETCH/WRITE PMC passes of x3 yolo11s, the per-op SQ table.  Every GPU step has its own limit; a failure stops it.
cd "$(dirname "$0")/.." || exit 1
R="$PWD"
O=gpurun_out/j
mkdir -p $O
export TMPDIR=/tmp
b() {  # name, bench args
  local n=$1; shift
  echo "[j] bench $n $(date +%T)"
  timeout -k 10 420 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['value'], d['device_images_per_s'], d.get('parity',{}).get('meets_tolerance'))"
}
b s_x3
b n_x3 --model n
b seg_x3 --model s --task segment --batch 4
echo "[j] prof $(date +%T)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- \
  python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline > "$R/$O/prof.log" 2>&1 || { tail -20 "$R/$O/prof.log"; exit 1; }
echo "[j] pmc $(date +%T)"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch_s_x3" -o run -- \
  python3 "$R/tools/pmc_forward.py" --model s --dtype x3 > "$R/$O/pmc_fetch_s_x3.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write_s_x3" -o run -- \
  python3 "$R/tools/pmc_forward.py" --model s --dtype x3 > "$R/$O/pmc_write_s_x3.log" 2>&1 || exit $?
cd "$R"
echo "[j] sq $(date +%T)"
bash tools/gpu_sq_table.sh r03j_s_b8_x3 --model s --dtype x3 || exit $?
echo "[j] done $(date +%T)"
echo "[j] suite $(date +%T)"
bash tools/gpu_suite.sh || exit $?
echo "[j] suite done $(date +%T)"
