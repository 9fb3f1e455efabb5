#!/bin/bash
# Round-5 A/B of HIP's kernel-argument placement (HIP_FORCE_DEV_KERNARG: 1 = device memory, 0 = host memory, unset =
# the runtime's default) on the headline bench, interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05ae}
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
for rep in 1 2; do
  for v in unset 1 0; do
    if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
    run "bench_${v}_$rep" 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-roofline --no-f16
  done
done
unset HIP_FORCE_DEV_KERNARG
echo done >> "$OUT/steps.log"
