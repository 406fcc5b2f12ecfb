#!/bin/bash
# Wave-cycle breakdown of one headline frame (run through gpurun):
#   pass "wait": SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt) + SQ_WAIT_INST_ANY
#                (issue stall) + SQ_ACTIVE_INST_ANY (MI355X_MICROARCH.md, PMC table)
#   pass "sqc":  scalar data / instruction cache hits and misses
# Summaries land in gpurun_out/stall_<tag>/.   tools/stall_profile.sh <tag> [ab_flags args]
set -e
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/stall_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
args="$*"; [ -z "$args" ] && args="--reps 1 ACCEL_BVH"
P="$GRAFT_REPO_ROOT/tools/ab_flags.py $args"
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VALU --output-format csv -d $out/wait -o wait -- python3 $P > $out/wait.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $out/sqc -o sqc -- python3 $P > $out/sqc.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/pmc_traffic.py $out/wait $out/sqc --kernel "${KERNEL:-render_kernel<false, false, true, false, true>}" --out $out/summary.json
echo done
