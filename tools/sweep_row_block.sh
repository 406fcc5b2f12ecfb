#!/bin/bash
# Slowest rank of the headline frame's 1/8 share per band height (rows per
# interleaved band), pilot order (GPU box):  tools/sweep_row_block.sh [rb ...]
for rb in ${@:-8 4 2 1}; do
  timeout -k 10 120 python tools/rank_share.py --preset c2 --world 8 --rank 0 1 2 3 4 5 6 7 --reps 2 \
    --row-block $rb --flags PILOT_SCHEDULE 2>/dev/null | python3 -c "
import json,sys
r=[json.loads(l) for l in sys.stdin if l.startswith('{')]
t={}
for x in r: t.setdefault(x['rank'],[]).append(x['kernel_ms'])
m={k:min(v) for k,v in t.items()}
print('row_block', $rb, 'per-rank min ms', [m[k] for k in sorted(m)], 'max', max(m.values()), 'segments', sum(x['segments'] for x in r)//2)" || exit 1
done
