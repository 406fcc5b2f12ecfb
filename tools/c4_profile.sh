#!/bin/bash
# Counter evidence for one rank's share of a BASELINE config (GPU box, through
# gpurun).  Default: the C4 rank-0 share (16384^2 / 8 ranks, 10 001 spheres) at
# a reduced spp, and the headline frame at the same spp for comparison.
#   tools/c4_profile.sh <tag> [spp] [cases]
# cases: space-separated among c4g (C4 share, grid in global memory), c4c (C4
# share, cells in LDS), c2 (headline frame, whole grid in LDS); default all.
# Leaves in gpurun_out/c4prof_<tag>/: work counters, kernel trace, and PMC
# passes (SQ issue/lane use, wave-cycle split, L1/L2 (TCP/TCC) reads, FETCH_SIZE)
# summarised by tools/pmc_traffic.py into <case>_summary.json.
set -e
tag=$1; spp=${2:-100}; cases=${3:-"c4g c4c c2"}
out=$GRAFT_REPO_ROOT/gpurun_out/c4prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/tools/rank_share.py
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
for case in $cases; do
  case $case in
    c4g) A="--preset c4 --world 8 --rank 0 --spp $spp --grid-mode global";;
    c4c) A="--preset c4 --world 8 --rank 0 --spp $spp --grid-mode cells";;
    *) A="--preset c2 --world 1 --rank 0 --spp $spp";;
  esac
  timeout -k 10 300 python3 $R $A --reps 2 --count-work > $out/${case}_work.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${case}_kt -o kt -- python3 $R $A > $out/${case}_kt.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $out/${case}_sq -o sq -- python3 $R $A > $out/${case}_sq.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d $out/${case}_wait -o wait -- python3 $R $A > $out/${case}_wait.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/${case}_tcp -o tcp -- python3 $R $A > $out/${case}_tcp.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/${case}_fetch -o fetch -- python3 $R $A > $out/${case}_fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES --output-format csv -d $out/${case}_sqc -o sqc -- python3 $R $A > $out/${case}_sqc.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_LDS --output-format csv -d $out/${case}_lds -o lds -- python3 $R $A > $out/${case}_lds.log 2>&1
done
cd $GRAFT_REPO_ROOT
for case in $cases; do
  python3 tools/pmc_traffic.py $out/${case}_sq $out/${case}_wait $out/${case}_tcp $out/${case}_fetch $out/${case}_sqc $out/${case}_lds \
    --kernel "${KERNEL:-render_kernel<false, false, true, false, true}" --workload "$case share spp=$spp" \
    --out $out/${case}_summary.json > /dev/null
done
echo done
