#!/bin/bash
# A/B of launch-plan variants (build/variants/<name>.so, "base" = in-tree) on
# C3's whole frame and C4's rank-0 share (GPU box); base first and last.
#   tools/ab_launch_plans.sh <name> ...
set -e
run() {
  local lib=ray-tracing-in-one-weekend_amd/librtow.so
  [ "$1" != base ] && lib=build/variants/$1.so
  echo "$1 c3 $(RTOW_LIB=$lib timeout -k 10 120 python bench.py --preset c3 --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["lane_efficiency"])')"
  echo "$1 c4share $(RTOW_LIB=$lib timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --flags PILOT_SCHEDULE 2>/dev/null | tail -1)"
}
run base
for v in "$@"; do run $v; done
run base
