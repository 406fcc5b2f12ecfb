#!/bin/bash
# Headline frame kernel time per layer-grid cell scale (whole grid in LDS)
set -e
mkdir -p gpurun_out
for g in 1.0 1.02 1.04 1.06 1.08 1.1 1.12 1.14 1.16 1.18 1.2 1.22 1.24 1.26 1.28 1.3 1.32 1.34 1.0; do
  timeout -k 10 120 python tools/ab_flags.py --reps 2 --option GRID_SCALE=$g ACCEL_BVH+PILOT_SCHEDULE 2>/dev/null | sed "s/^/scale $g /" >> gpurun_out/r04z2_sweep_c2.log
done
echo done
