#!/bin/bash
# PMC summaries of rank 0's 1/N share of the headline frame (GPU box, through
# gpurun), for bench.py's N > 1 lines: the same passes as profile_round.sh
# (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ) over tools/rank_share.py with the
# bench's flags (layer grid, pilot schedule, automatic units).  Summaries in
# gpurun_out/share_<tag>/w<N>/pmc_traffic.json (copy to
# profiles/pmc_traffic_bvh_w<N>.json).
#   tools/profile_shares.sh <tag> [worlds...]
set -e
tag=$1; shift
worlds=${*:-"2 4 8"}
WL="final random-spheres scene 3840x2160 @ 500spp depth 50"
K=${KERNEL:-"render_kernel<false, false, true, false, true, 1, false>"}
for w in $worlds; do
  out=$GRAFT_REPO_ROOT/gpurun_out/share_$tag/w$w
  mkdir -p $out
  cd /tmp && export TMPDIR=/tmp
  R="$GRAFT_REPO_ROOT/tools/rank_share.py --preset c2 --world $w --rank 0 --flags PILOT_SCHEDULE --reps 4"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $R > $out/kt.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $R > $out/fetch.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $R > $out/write.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $out/sq -o sq -- python3 $R > $out/sq.log 2>&1
  cd $GRAFT_REPO_ROOT
  python3 tools/pmc_traffic.py $out/fetch $out/write $out/sq --kernel "$K" --world $w --workload "$WL" \
    --out $out/pmc_traffic.json > /dev/null
done
echo done
