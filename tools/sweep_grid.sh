#!/bin/bash
# Grid cell size sweep (GPU box): RTOW_GRID_SCALE scales the layer grid's cell
# side (1 = about one sphere per cell).  tools/sweep_grid.sh <lib> <scale> ...
set -e
lib=$1; shift
for s in "$@"; do
  RTOW_GRID_SCALE=$s RTOW_LIB=$lib timeout -k 10 90 python tools/ab_flags.py --reps 2 ACCEL_BVH+PILOT_SCHEDULE | sed "s/^/scale=$s /"
done
