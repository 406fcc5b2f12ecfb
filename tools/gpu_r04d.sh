# round 4: A/B xg (micro set without compaction) / xd; C4 xf (cross-cell item prefetch);
# PC sampling availability and a first stochastic profile
bash tools/gpu_steps.sh \
  "r04d_ab|500|REPS=3 bash tools/ab_libs.sh xg xd" \
  "r04d_ab_c4|500|bash tools/ab_c4.sh xd xf" \
  "r04d_pcs_list|60|cd /tmp && rocprofv3 -L" \
  "r04d_pcs|200|bash tools/pc_sample.sh r04d stochastic cycles 1048576"
