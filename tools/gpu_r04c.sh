# round 4: headline A/B of the compacted extras (xc2), the micro set (xd) and
# dielectric parking (xp4, xp12); C4 share A/B of the pipelined item loads (xe)
bash tools/gpu_steps.sh \
  "r04c_ab|600|REPS=3 bash tools/ab_libs.sh xc2 xd xp4 xp12" \
  "r04c_ab_c4|500|bash tools/ab_c4.sh xd xe"
