# full GPU round: all GPU tests, f16 + i8 bench lines, rocprof kernel stats of the f16 and i8 bench commands
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp YM_TUNE_DIR="$PWD/gpurun_out/tune"
bash tools/gpu_round.sh tests bench bench_i8 && \
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_i8" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --dtype i8 --steps 50 --warmup 10 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_i8.log" 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1; echo prof rc=$?
