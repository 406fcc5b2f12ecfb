# round 4: xq (DDA step before exit + one wait + 32-bit offsets), xr (+ one u16
# entry per cell: first-item address | count, empty cells list a dummy item:
# no empty-cell branch), xt (+ NaN-keyed candidate: one select for the t_min test)
bash tools/gpu_steps.sh \
  "r04l_ab|500|REPS=3 bash tools/ab_libs.sh xr xt xu"
