#!/bin/bash
# Kernel time of the headline frame under builder env knobs (GPU box):
#   tools/sweep_env.sh "RTOW_BVH_LEAF=2 RTOW_BVH_COLLAPSE=0.3" "..." ...
# ("-" = defaults).  Each line is one ab_flags run (2 reps, image sha256).
mkdir -p gpurun_out
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  echo -n "[$e] "
  env $e timeout -k 10 90 python tools/ab_flags.py --reps 2 ACCEL_BVH || exit $?
done
