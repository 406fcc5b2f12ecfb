#!/bin/bash
# Kernel ms per rt_params.units (waves per tile) with the pilot schedule, for
# C1 on one GPU and the 1/4, 1/8 shares of the headline frame and C3 (GPU box):
#   tools/sweep_units.sh [units ...]   (0 = the automatic choice)
for u in ${@:-0 1 2 3 4 5 6 8}; do
  for cfg in "c1 1" "c2 4" "c2 8" "c3 8"; do
    set -- $cfg
    timeout -k 10 120 python tools/rank_share.py --preset $1 --world $2 --rank 0 --reps 3 --units $u \
      --flags PILOT_SCHEDULE 2>/dev/null | tail -2 | python3 -c "
import json,sys
r=[json.loads(l) for l in sys.stdin if l.startswith('{')]
print('units', $u, '$1/$2', [x['kernel_ms'] for x in r])" || exit 1
  done
done
