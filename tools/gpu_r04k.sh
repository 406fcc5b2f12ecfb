# round 4: DDA step before the exit test (xn), + one wait for the cell range (xo),
# + 32-bit offsets for the turn-table and shading-record loads (xq)
bash tools/gpu_steps.sh \
  "r04k_ab|500|REPS=3 bash tools/ab_libs.sh xn xo xq"
