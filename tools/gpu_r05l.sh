#!/bin/bash
# Round-5 x3 split configurations on 128-wide tiles (csrc/ym_conv_dma.hip YM_DMA_X3_CFGS ids 9-13 = op cfgs 127-131):
# a fresh ym_tune of the 40² / 20² ops (tools/retable.py, YM_RETABLE_OPS; per-candidate log), a table that takes a
# fresh pick only where it is one of the new configurations (every other op keeps its committed, in-context cfg), then
# a same-box A/B against the committed table: per-op replay tables and bench lines, interleaved.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r05l}
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
OPS="model.5,model.6.cv1,model.6.m.0.cv1+cv2,model.6.m.0.m.0.cv1+cv2,model.6.m.0.m.1.cv1+cv2,model.6.m.0.cv3,model.6.cv2,model.7,model.8.cv1,model.8.m.0.cv1+cv2,model.8.m.0.m.0.cv1,model.8.m.0.m.0.cv2,model.8.m.0.m.1.cv1,model.8.m.0.m.1.cv2,model.8.m.0.cv3,model.8.cv2,model.9.cv1,model.9.cv2,model.10.cv1,model.10.m.0.attn.qkv,model.10.m.0.attn.proj,model.10.m.0.ffn.0,model.10.m.0.ffn.1,model.10.cv2,model.13.cv1,model.13.m.0.cv1,model.13.m.0.cv2,model.13.cv2,model.17,model.19.cv1,model.19.m.0.cv1,model.19.m.0.cv2,model.19.cv2,model.20,model.22.cv1,model.22.m.0.cv1+cv2,model.22.m.0.m.0.cv1,model.22.m.0.m.0.cv2,model.22.m.0.m.1.cv1,model.22.m.0.m.1.cv2,model.22.m.0.cv3,model.22.cv2,model.23.cv2.1.0,model.23.cv2.1.1+2,model.23.cv3.1.0.1,model.23.cv3.1.1.1+2,model.23.cv2.2.0,model.23.cv2.2.1+2,model.23.cv3.2.0.1,model.23.cv3.2.1.1+2"
for step in ${STEPS:-retable mix ab}; do
  case $step in
    retable) YM_RETABLE_OPS="$OPS" YM_TUNE_LOG=1 run retable 600 python -u tools/retable.py s:detect:x3:8 ;;
    mix) mkdir -p "$OUT/tune" && python3 - "$OUT" <<'PY' > "$OUT/mix.log" 2>&1 || exit 1
import json, sys
out = sys.argv[1]
name = "s-detect-x3-b8-640x640.json"
com = json.load(open("yolo-infer_amd/yolomi/tuned/" + name))
fresh = json.load(open("gpurun_out/tuned/" + name))
assert com["ops"] == fresh["ops"]
NEW = set(range(127, 132))
def uses_new(c):
    if c >= 1 << 20:
        c -= 1 << 20
        return (c >> 8) in NEW or (c & 255) in NEW
    return c in NEW
cfg = [f if uses_new(f) else c for c, f in zip(com["cfg"], fresh["cfg"])]
for n, c, f in zip(com["ops"], com["cfg"], fresh["cfg"]):
    if uses_new(f):
        print(f"{n}: committed {c} -> {f}")
t = dict(com, cfg=cfg, note="r05l: committed table + the new 128-wide x3 split configs where the fresh tune picked them")
json.dump(t, open(f"{out}/tune/{name}", "w"))
PY
      echo "[mix] rc=0" >> "$OUT/steps.log" ;;
    ab)
      for rep in 1 2; do
        for v in new com; do
          if [ $v = new ]; then export YM_TUNE_DIR=$OUT/tune YM_PREFER_CACHE=1; else unset YM_TUNE_DIR YM_PREFER_CACHE; fi
          run "optable_${v}_$rep" 200 python -u tools/op_table.py --model s --dtype x3
          run "bench_${v}_$rep" 300 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-roofline --no-f16
        done
      done ;;
  esac
done
echo done >> "$OUT/steps.log"
