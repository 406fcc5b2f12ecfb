# round 4: packed cell entries (xr), independent material blocks (xw), both (xrw)
bash tools/gpu_steps.sh \
  "r04m_ab|600|REPS=3 bash tools/ab_libs.sh xr xw xrw xr xw xrw"
