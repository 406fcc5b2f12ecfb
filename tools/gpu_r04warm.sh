#!/bin/bash
# (run while bench.py, rank_share.py and rank_times.py tuned the grid by default; they now need
#  --grid-tune for that, and --no-grid-tune is gone: the untuned runs are the default)
# Is the tuned bench's gain the grid or the extra GPU work before the warmup?
set -e
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 10"
for k in 1 2; do
  timeout -k 10 300 $B --warmup 2 --no-grid-tune | sed "s/^/notune_w2 /" >> gpurun_out/r04warm.log 2>&1
  timeout -k 10 300 $B --warmup 8 --no-grid-tune | sed "s/^/notune_w8 /" >> gpurun_out/r04warm.log 2>&1
  timeout -k 10 300 $B --warmup 2 | sed "s/^/tune_w2 /" >> gpurun_out/r04warm.log 2>&1
done
for g in 1.0 1.11 1.22 1.0 1.11 1.22; do
  timeout -k 10 120 python tools/ab_flags.py --reps 4 --option GRID_SCALE=$g ACCEL_BVH+PILOT_SCHEDULE 2>/dev/null | sed "s/^/scale $g /" >> gpurun_out/r04warm_ab.log
done
echo done
