#!/bin/bash
# C4's rank-0 share at reduced spp (GPU box): the automatic placement (cell
# starts in LDS, items from L1, the fitted cell size) against the grid read
# wholly from global memory at finer cell scales, which the LDS placement
# cannot hold.  One line per configuration: the
# rank_share.py JSON with its work counters.
SPP=${SPP:-200}
run() {
  out=$(timeout -k 10 150 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp $SPP --flags PILOT_SCHEDULE --reps 2 --count-work $2 2>/dev/null) || exit 1
  echo "$out" | sed "s/^/$1 /"
}
run auto "--grid-mode auto"
for g in ${SCALES:-0.6 0.7 0.8 0.9 1.0 1.1 1.17}; do
  run "global_$g" "--grid-mode global --grid-scale $g"
done
run auto "--grid-mode auto"
