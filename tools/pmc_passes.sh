#!/bin/bash
# Extra PMC passes over one headline frame (GPU box): SMEM latency, dual VALU
# issue and the VALU instruction mix.  Summaries in gpurun_out/pmc_<tag>/.
#   tools/pmc_passes.sh <tag>
set -e
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/tools/ab_flags.py --reps 1 ACCEL_BVH"
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_SMEM_NORM SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_BUSY_CU_CYCLES --output-format csv -d $out/a -o a -- python3 $P > $out/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $out/b -o b -- python3 $P > $out/b.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/pmc_traffic.py $out/a $out/b --kernel "${KERNEL:-render_kernel<false, false, true, false, true>}" --out $out/summary.json
echo done
