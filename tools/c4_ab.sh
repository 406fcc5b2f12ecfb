#!/bin/bash
# A/B of the C4 rank-0 share (GPU box): launch order vs pilot order, units,
# and a build without the far-origin scan fallback (timing only: that build
# can differ from the scan).  gpurun_out/c4ab_<tag>.log
tag=$1; spp=${2:-100}
R="python3 tools/rank_share.py --preset c4 --world 8 --rank 0 --spp $spp --reps 2"
out=gpurun_out/c4ab_$tag.log
mkdir -p gpurun_out; : > $out
run() { echo "== $*" >> $out; timeout -k 10 120 "$@" 2>/dev/null | grep '^{' >> $out || exit 1; }
run $R --grid-mode global
run $R --grid-mode global --flags PILOT_SCHEDULE
run $R --grid-mode global --units 8
run $R --grid-mode global --units 8 --flags PILOT_SCHEDULE
RTOW_LIB=build/variants/noscanall.so run $R --grid-mode global
RTOW_LIB=build/variants/noscanall.so run $R --grid-mode global --flags PILOT_SCHEDULE
run python3 tools/rank_share.py --preset c2 --world 1 --rank 0 --spp $spp --reps 2
RTOW_LIB=build/variants/noscanall.so run python3 tools/rank_share.py --preset c2 --world 1 --rank 0 --spp $spp --reps 2
cat $out
