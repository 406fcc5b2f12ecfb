# round 4: marginal cost of scalar vs vector instructions in the grid item loop
# (probe builds: +2 / +5 SALU or +1-2 VALU per item iteration, same image)
bash tools/gpu_steps.sh \
  "r04j_ab|500|REPS=3 bash tools/ab_libs.sh xs1 xs4 xv1"
