# round 4: independent material blocks (xw, re-linked with the kparams extras
# pointers) vs the same plus host-resolved extras pointers, no layer-mode test
# in the grid build, no explicit ballot before the ground's sequence (xz)
bash tools/gpu_steps.sh \
  "r04n_ab|600|REPS=3 bash tools/ab_libs.sh xw xz xa xw xz xa"
