#!/bin/bash
# Same-box A/B of the x3 epilogue store pattern (YM_PAIRST bit mask: 1 LDS-DMA, 2 streaming, 4 stem, 8 fused
# Bottleneck lane-pair whole-chunk stores; 0 = per-lane 8-byte pieces everywhere): per-op replay tables of yolo11s
# B=8 x3 for every mask, twice, interleaved; then the bench line for 0 / 15, twice.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/ab
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/permlane_probe tools/permlane_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/permlane_probe | tee $O/permlane_probe.txt || exit 1
for r in 1 2; do
  for p in 0 15 1 2 4 8; do
    YM_PAIRST=$p timeout -k 10 300 python -u tools/op_table.py --model s --dtype x3 > $O/op_s_p${p}_r$r.txt 2>&1 || { tail -20 $O/op_s_p${p}_r$r.txt; exit 1; }
    echo "pairst=$p run $r: $(tail -1 $O/op_s_p${p}_r$r.txt)"
  done
done
for r in 1 2; do
  for p in 0 15; do
    YM_PAIRST=$p timeout -k 10 400 python bench.py --no-cpu --no-f16 > $O/bench_p${p}_r$r.json 2> $O/bench_p${p}_r$r.err || { tail -20 $O/bench_p${p}_r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_p${p}_r$r.json'));print('pairst=$p bench', d['value'], d['device_images_per_s'], d['ms_per_step'])"
  done
done
