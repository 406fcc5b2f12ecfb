#!/bin/bash
# A/B kernel time of alternative librtow builds on the headline frame (GPU box):
#   tools/ab_libs.sh <name> ...   (build/variants/<name>.so; "base" = the in-tree build)
# Runs base first and last to bracket drift; each run checks the image sha256.
# (.gpurunignore keeps build/variants off the GPU box: drop that line for an A/B call.)
set -e
mkdir -p gpurun_out
run() {
  local lib=ray-tracing-in-one-weekend_amd/librtow.so
  [ "$1" != base ] && lib=build/variants/$1.so
  RTOW_LIB=$lib timeout -k 10 90 python tools/ab_flags.py --reps ${REPS:-2} ${AB_FLAGS:-ACCEL_BVH+PILOT_SCHEDULE} | sed "s/^/$1 /"
}
run base
for v in "$@"; do run $v; done
run base
