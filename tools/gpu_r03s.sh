bash tools/gpu_steps.sh \
  "r03s_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03s_ab|400|REPS=3 bash tools/ab_libs.sh prepersist"
