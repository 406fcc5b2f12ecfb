#!/bin/bash
# A/B of the C4 rank-0 share (1/8 of 16384^2, 10 001 spheres) at SPP samples per
# pixel (default 200) for alternative librtow builds (GPU box):
#   tools/ab_c4.sh <name> ...   (build/variants/<name>.so; "base" = the in-tree build)
# base runs first and last to bracket drift.
# (.gpurunignore keeps build/variants off the GPU box: drop that line for an A/B call.)
set -e
spp=${SPP:-200}
run() {
  local lib=ray-tracing-in-one-weekend_amd/librtow.so
  [ "$1" != base ] && lib=build/variants/$1.so
  echo "$1 $(RTOW_LIB=$lib timeout -k 10 150 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp $spp --reps ${REPS:-2} --flags PILOT_SCHEDULE 2>/dev/null | grep '^{' | tail -1)"
}
run base
for v in "$@"; do run $v; done
run base
