#!/bin/bash
# per-stage slope / fixed intercept of the LDS-DMA conv: µs per launch vs K at a 20x20 (M = 3200) and 40x40 map
cd "$(dirname "$0")/.." || exit 1
for cfg in "$@"; do
  for C in 64 128 256 512 1024; do
    timeout -k 5 60 ./tools/dma_probe_ns 8 20 20 $C 64 3 $cfg | head -1 || exit 1
  done
done
