#!/bin/bash
# One GPU-box session: GPU parity tests, the bench line, a rocprofv3 kernel-trace/stats run of the same bench
# command, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) of tools/pmc_forward.py.  Every GPU step has its
# own time limit; after a fault / abort / timeout nothing further runs on the GPU.
#   bash tools/gpu_round.sh [tests|bench|prof|pmc|optable ...]   (default: tests bench prof pmc)
# BENCH_ARGS / PMC_ARGS / OPT_ARGS: extra arguments of the prof-step bench, tools/pmc_forward.py, tools/op_table.py
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp YM_TUNE_DIR="$PWD/gpurun_out/tune"
steps=("$@"); [ ${#steps[@]} -eq 0 ] && steps=(tests bench prof pmc)
fatal() { local rc=$1; [ "$rc" -eq 124 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
for s in "${steps[@]}"; do
  echo "[gpu_round] step $s $(date +%T)"
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gt.log 2>&1; rc=$?
           tail -15 gpurun_out/gt.log ;;
    qtests) timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/qt.log 2>&1; rc=$?
           tail -25 gpurun_out/qt.log ;;
    bench_i8) timeout -k 10 500 python bench.py --dtype i8 > gpurun_out/bench_i8.json 2> gpurun_out/bench_i8.err; rc=$?
           cat gpurun_out/bench_i8.json; tail -3 gpurun_out/bench_i8.err ;;
    bench) timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
           cat gpurun_out/bench.json ;;
    bench_s) timeout -k 10 400 python bench.py --model s > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err; rc=$?
           cat gpurun_out/bench_s.json ;;
    prof)  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 \
             --warmup 10 --no-cpu --no-f16 $BENCH_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1; rc=$?; cd "$GRAFT_REPO_ROOT" ;;
    pmc)   cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pmc_forward.py" $PMC_ARGS \
             > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log" 2>&1; rc=$?
           if [ $rc -eq 0 ]; then timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pmc_forward.py" $PMC_ARGS \
             > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log" 2>&1; rc=$?; fi
           cd "$GRAFT_REPO_ROOT" ;;
    optable) timeout -k 10 300 python -u tools/op_table.py $OPT_ARGS > gpurun_out/op_table.txt 2>&1; rc=$?
           tail -3 gpurun_out/op_table.txt ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "[gpu_round] step $s rc=$rc $(date +%T)"
  if fatal $rc; then echo "[gpu_round] fatal rc=$rc in $s: stopping"; exit $rc; fi
  if [ "$rc" -ne 0 ]; then any_fail=$rc; fi
done
exit ${any_fail:-0}
