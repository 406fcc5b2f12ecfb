#!/bin/bash
# C4 rank-0 share per cell scale, three interleaved passes (noise vs shape)
set -e
mkdir -p gpurun_out
for pass in 1 2 3; do
  SCALES="1.113 1.15 1.16 1.17 1.18 1.19 1.2 1.21" SPP=200 bash tools/sweep_scale_c4.sh >> gpurun_out/r04x_sweep_c4.log 2>&1
done
echo done
