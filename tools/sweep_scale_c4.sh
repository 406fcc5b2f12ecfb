#!/bin/bash
# C4 rank-0 share (reduced spp) per layer-grid cell scale (GPU box)
for g in ${SCALES:-0.8 1.0 1.25 1.5}; do
  echo "scale $g $(timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp ${SPP:-200} --grid-scale $g 2>/dev/null | tail -1)" || exit 1
done
