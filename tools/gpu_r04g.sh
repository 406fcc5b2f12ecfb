# round 4: C4 share A/B of 12-byte item reads with the tie key read by candidates only (xm)
bash tools/gpu_steps.sh \
  "r04g_ab_c4|500|bash tools/ab_c4.sh xm xm"
