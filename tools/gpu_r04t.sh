# round 4: C4 rank-0 share at 200 spp: saddr item loads (xc4), two items per iteration (xc5)
bash tools/gpu_steps.sh \
  "r04t_ab_c4|600|bash tools/ab_c4.sh xc4 xc5 xc4 xc5"
