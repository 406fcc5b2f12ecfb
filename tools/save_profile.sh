#!/bin/bash
# Copy one GPU run's results (tools/gpu_steps.sh tests/bench + tools/profile_round.sh <tag>)
# from gpurun_out/ into profiles/<tag>_* and make its PMC summary the bench's
# (profiles/pmc_traffic_bvh.json, keyed to the kernel source it was collected on).
#   tools/save_profile.sh <tag>
set -e
tag=$1
P=gpurun_out/prof_$tag
cp $P/kt/kt_kernel_stats.csv profiles/${tag}_kernel_stats.csv
cp $P/kt/kt_kernel_trace.csv profiles/${tag}_kernel_trace.csv
cp $P/sq/sq_counter_collection.csv profiles/${tag}_pmc_sq.csv
cp $P/fetch/fetch_counter_collection.csv profiles/${tag}_pmc_fetch.csv
cp $P/write/write_counter_collection.csv profiles/${tag}_pmc_write.csv
cp $P/pmc_traffic.json profiles/pmc_traffic_bvh.json
[ -f gpurun_out/tests.log ] && cp gpurun_out/tests.log profiles/${tag}_gpu_tests.log
[ -f gpurun_out/bench.log ] && grep -v amdgpu.ids gpurun_out/bench.log > profiles/${tag}_bench.log
python3 tools/kernel_trace_avg.py profiles/${tag}_kernel_trace.csv
