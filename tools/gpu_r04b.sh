# round 4, session 2: counters of the current device code (full frame + 1/2, 1/4, 1/8 shares),
# and the compacted extras root sequences (variant xc) against the in-tree build
bash tools/gpu_steps.sh \
  "bench|300|python bench.py --steps 20 --warmup 5" \
  "ab_xc|400|REPS=3 bash tools/ab_libs.sh xc" \
  "prof|900|bash tools/profile_round.sh r04b" \
  "shares|900|bash tools/profile_shares.sh r04b 2 4 8"
