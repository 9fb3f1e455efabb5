#!/bin/bash
# Same-box A/B of two builds of the library (abso/old.so vs abso/new.so), alternating, then the new one restored.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-ab_so}
mkdir -p "$OUT"
for v in old new old new; do
  n=$((n + 1))
  cp abso/$v.so yolo-infer_amd/yolomi/libyolomi.so
  timeout -k 10 300 python -u bench.py --no-roofline --steps ${STEPS:-300} $ARGS > "$OUT/ab_${v}_$n.log" 2>&1
  rc=$?
  echo "[$v] rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then break; fi
done
cp abso/new.so yolo-infer_amd/yolomi/libyolomi.so
exit $rc
