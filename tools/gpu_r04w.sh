#!/bin/bash
# Grid cell-scale sweeps on the final build: C4 rank-0 share (cells in LDS)
# and the headline frame (whole grid in LDS).
set -e
mkdir -p gpurun_out
SCALES="1.15 1.18 1.2 1.22 1.25 1.27 1.113 1.2" SPP=200 bash tools/sweep_scale_c4.sh > gpurun_out/r04w_sweep_c4.log 2>&1
for g in 1.0 1.05 1.1 1.15 1.2 1.0; do
  timeout -k 10 120 python tools/ab_flags.py --reps 2 --option GRID_SCALE=$g ACCEL_BVH+PILOT_SCHEDULE >> gpurun_out/r04w_sweep_c2.log 2>&1
done
echo done
