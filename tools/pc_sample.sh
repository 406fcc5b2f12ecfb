#!/bin/bash
# PC sampling of one headline frame (GPU box): rocprofv3's stochastic (or
# host-trap) PC sampler over tools/ab_flags.py, for a per-instruction profile
# of the render kernel.  Output in gpurun_out/pcs_<tag>/.
#   tools/pc_sample.sh <tag> <method> <unit> <interval> [lib]
set -e
tag=$1; method=$2; unit=$3; interval=$4; lib=${5:-ray-tracing-in-one-weekend_amd/librtow.so}
out=$GRAFT_REPO_ROOT/gpurun_out/pcs_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
RTOW_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $method \
  --pc-sampling-unit $unit --pc-sampling-interval $interval --output-format csv -d $out -o pcs -- \
  python3 $GRAFT_REPO_ROOT/tools/ab_flags.py --reps 1 ACCEL_BVH+PILOT_SCHEDULE > $out/run.log 2>&1
ls -la $out
