#!/bin/bash
# A/B of the C4 rank-0 share (GPU box): grid placement (global / cells in
# LDS), units and launch order vs pilot order; the headline frame for
# comparison.  gpurun_out/c4ab_<tag>.log
tag=$1; spp=${2:-100}
R="python3 tools/rank_share.py --preset c4 --world 8 --rank 0 --spp $spp --reps 2"
out=gpurun_out/c4ab_$tag.log
mkdir -p gpurun_out; : > $out
run() { echo "== $*" >> $out; timeout -k 10 120 "$@" 2>/dev/null | grep '^{' >> $out || exit 1; }
for mode in global cells; do
  run $R --grid-mode $mode
  run $R --grid-mode $mode --flags PILOT_SCHEDULE
  run $R --grid-mode $mode --units 2
  run $R --grid-mode $mode --units 4 --flags PILOT_SCHEDULE
done
run python3 tools/rank_share.py --preset c2 --world 1 --rank 0 --spp $spp --reps 2
cat $out
