# round 4: xzab / xzabc vs + flat pool take (xzabcd) vs + folded uniform scales and
# lens-conditional draw (xze)
bash tools/gpu_steps.sh \
  "r04p_ab|700|REPS=3 bash tools/ab_libs.sh xzabc xzabcd xze xzabr xzabc xzabcd xze xzabr"
