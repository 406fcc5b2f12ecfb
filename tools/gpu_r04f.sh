# round 4: A/B of the folded uniform scales + lens-conditional draw (xk)
bash tools/gpu_steps.sh \
  "r04f_ab|400|REPS=3 bash tools/ab_libs.sh xk xk"
