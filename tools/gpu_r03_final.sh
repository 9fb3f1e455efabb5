#!/bin/bash
# Round-3 final evidence: bench lines of every BASELINE config on its default (x3) plan plus the int8 / fp8 / f32
# plans, rocprofv3 kernel stats of the headline bench command, FETCH/WRITE PMC passes (x3 yolo11s, int8 yolo11n),
# the per-op SQ table of the headline workload.  Every GPU step has its own limit; a failure stops the script.
cd "$(dirname "$0")/.." || exit 1
R="$PWD"
O=gpurun_out/fin
mkdir -p $O
export TMPDIR=/tmp
b() {  # name, bench args
  local n=$1; shift
  echo "[fin] bench $n $(date +%T)"
  timeout -k 10 420 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$n.json'));print('$n', d['value'], d['device_images_per_s'], d.get('parity',{}).get('meets_tolerance'))"
}
b s_x3
b n_x3 --model n
b seg_x3 --model s --task segment --batch 4
b n_i8 --model n --dtype i8
b n_f8 --model n --dtype f8
b s_f32 --dtype f32 --steps 50 --warmup 5 --no-cpu
echo "[fin] prof $(date +%T)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- \
  python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --no-f16 --no-roofline > "$R/$O/prof.log" 2>&1 || { tail -20 "$R/$O/prof.log"; exit 1; }
echo "[fin] pmc $(date +%T)"
for cfg in "s x3" "n i8"; do
  set -- $cfg
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/pmc_fetch_$1_$2" -o run -- \
    python3 "$R/tools/pmc_forward.py" --model $1 --dtype $2 > "$R/$O/pmc_fetch_$1_$2.log" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/pmc_write_$1_$2" -o run -- \
    python3 "$R/tools/pmc_forward.py" --model $1 --dtype $2 > "$R/$O/pmc_write_$1_$2.log" 2>&1 || exit $?
done
cd "$R"
echo "[fin] sq $(date +%T)"
bash tools/gpu_sq_table.sh r03e_s_b8_x3 --model s --dtype x3 || exit $?
echo "[fin] done $(date +%T)"
