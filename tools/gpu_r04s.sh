# round 4: branchless refine (xf2), + selects for the near-zero fallback and the
# path end (xf3)
bash tools/gpu_steps.sh \
  "r04s_ab|600|REPS=3 bash tools/ab_libs.sh xf2 xf3 xf4 xf5 xf2 xf3 xf4 xf5"
