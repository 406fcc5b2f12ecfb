#!/bin/bash
# Profile the default bench on the GPU box (run through gpurun) and leave the
# summaries under gpurun_out/prof_<tag>/:
#   kt     rocprofv3 --kernel-trace --stats   (per-kernel average duration)
#   fetch  --pmc FETCH_SIZE                   (separate passes: MI355X_MICROARCH HBM section)
#   write  --pmc WRITE_SIZE
#   sq     --pmc SQ_* instruction / cycle counters
# then tools/pmc_traffic.py -> gpurun_out/prof_<tag>/pmc_traffic.json.
#   tools/profile_round.sh <tag> [extra bench.py args]
set -e
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $B > $out/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $B --steps 3 > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $B --steps 3 > $out/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $out/sq -o sq -- python3 $B --steps 3 > $out/sq.log 2>&1
cd $GRAFT_REPO_ROOT
# the timed kernel: the LDS-resident layer grid build (bench default); KERNEL overrides
# (e.g. "render_kernel<false, false, true, false, false, 0>" for --accel layer_bvh)
K=${KERNEL:-"render_kernel<false, false, true, false, true, 1, false>"}
python3 tools/pmc_traffic.py $out/fetch $out/write $out/sq --kernel "$K" --world 1 \
  --workload "$(grep '"metric"' $out/kt.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["workload"])')" \
  --out $out/pmc_traffic.json
echo done
