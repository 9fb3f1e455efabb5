#!/bin/bash
# Lane-pair x3 stores, second A/B: the lane exchange by v_permlane*_swap (YM_PAIRST bit 16) — the permlane semantics
# probe, the x3 GPU tests under mask 31, then per-op replay tables and bench lines of yolo11s B=8 x3 for masks
# 0 / 5 / 15 / 21 / 31, interleaved twice.
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/ab2
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/permlane_probe tools/permlane_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/permlane_probe | tee $O/permlane_probe.txt || exit 1
grep -q "partner rule OK, permlane32_swap partner rule OK" $O/permlane_probe.txt || exit 3
YM_PAIRST=31 timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 300 --timeout-method thread > $O/x3_tests_31.log 2>&1 || { tail -40 $O/x3_tests_31.log; exit 1; }
tail -1 $O/x3_tests_31.log
for r in 1 2; do
  for p in 0 5 15 21 31; do
    YM_PAIRST=$p timeout -k 10 300 python -u tools/op_table.py --model s --dtype x3 > $O/op_s_p${p}_r$r.txt 2>&1 || { tail -20 $O/op_s_p${p}_r$r.txt; exit 1; }
    echo "pairst=$p run $r: $(tail -1 $O/op_s_p${p}_r$r.txt)"
  done
done
for r in 1 2; do
  for p in 0 5 15 21 31; do
    YM_PAIRST=$p timeout -k 10 400 python bench.py --no-cpu --no-f16 > $O/bench_p${p}_r$r.json 2> $O/bench_p${p}_r$r.err || { tail -20 $O/bench_p${p}_r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_p${p}_r$r.json'));print('pairst=$p bench', d['value'], d['device_images_per_s'], d['ms_per_step'])"
  done
done
