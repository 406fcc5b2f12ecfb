#!/bin/bash
# Headline kernel time under context options (GPU box), one ab_flags run per
# option set (2 reps, image sha256: every set must give the same image):
#   tools/sweep_options.sh "GRID_SCALE=1.1" "GRID_SCALE=1.0 GRID_PLACEMENT=3" "-" ...
# ("-" = defaults; names are include/rt.h's rt_option without RT_OPT_).
for set in "$@"; do
  args=()
  [ "$set" != "-" ] && for o in $set; do args+=(--option "$o"); done
  echo -n "[$set] "
  timeout -k 10 90 python tools/ab_flags.py --reps 2 "${args[@]}" ACCEL_BVH+PILOT_SCHEDULE || exit $?
done
