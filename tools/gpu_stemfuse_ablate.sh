#!/bin/bash
# fused stem phase ablations: rocprof kernel stats per YM_STEMFUSE_DBG value
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/r06g; mkdir -p $OUT; export TMPDIR=/tmp
for d in 0 1 2 4 8 16 31; do
  (cd /tmp && YM_STEMFUSE=1 YM_STEMFUSE_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/p$d" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu --no-f16 \
    --no-roofline > "$GRAFT_REPO_ROOT/$OUT/p$d.log" 2>&1) || exit $?
  echo "dbg $d done"
done
