# round 4: xz (material blocks + host-resolved extras pointers) + divergent main
# loop (xza) + row table with valid-column counts (xzab)
bash tools/gpu_steps.sh \
  "r04o_ab|600|REPS=3 bash tools/ab_libs.sh xz xza xzab xzabc xz xza xzab xzabc"
