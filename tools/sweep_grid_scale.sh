#!/bin/bash
# Headline kernel time per layer-grid cell scale (RTOW_GRID_SCALE, read at upload)
for g in ${SCALES:-0.9 1.0 1.1 1.2 1.35}; do
  echo "scale $g $(RTOW_GRID_SCALE=$g timeout -k 10 90 python tools/ab_flags.py --reps 2 ACCEL_BVH+PILOT_SCHEDULE)"
done
