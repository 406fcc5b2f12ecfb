#!/bin/bash
# Work counters of the C4 rank-0 share per cell scale (fast vs slow scales)
set -e
mkdir -p gpurun_out
for g in 1.15 1.16 1.17 1.18 1.2 1.21; do
  echo "scale $g $(timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp 100 --grid-scale $g --count-work 2>/dev/null | tail -1)" >> gpurun_out/r04y_c4_work.log
done
echo done
