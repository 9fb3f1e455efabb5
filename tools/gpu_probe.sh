#!/bin/bash
# Cycle-stamp probes of single LDS-DMA conv launches (tools/dma_probe.hip, built into tools/probe_bin/ on the CPU side):
# where the time of a 20x20 / 40x40 x3 conv goes (prologue, per-stage wait / barrier / issue / compute, epilogue).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
P=tools/probe_bin/dma_probe
o=gpurun_out/probe.log
: > $o
run() { echo "== $*" >> $o; timeout -k 5 60 env "$@" >> $o 2>&1 || { echo "rc=$?" >> $o; exit 1; }; }
# 3x3 128->128 at 20x20 B=8 (model.8.m.0.m.*): the tuned x3 config (DMA 13), a no-split one, and the f16 plan's
run PROBE_X3=1 $P 8 20 20 128 128 3 13
run PROBE_X3=1 $P 8 20 20 128 128 3 10
run PROBE_X3=1 $P 8 20 20 128 128 3 3
run PROBE_X3=0 $P 8 20 20 128 128 3 13
# 1x1 256->256 at 20x20 (model.8.m.0.cv1+cv2): DMA 12
run PROBE_X3=1 $P 8 20 20 256 256 1 12
run PROBE_X3=0 $P 8 20 20 256 256 1 12
# 3x3 256->256 at 40x40 s2 from 80x80 (model.5 is 128->256 s2: 80->40)
run PROBE_X3=1 $P 8 80 80 128 256 3 15 2
# cold-read layouts of the input max (csrc/ym_misc.hip input_stats)
echo "== read_probe" >> $o; timeout -k 5 60 tools/probe_bin/read_probe >> $o 2>&1 || { echo "rc=$?" >> $o; exit 1; }
echo done >> $o
