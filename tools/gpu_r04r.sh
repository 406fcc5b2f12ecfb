# round 4: kparams regrouped by use site (kpr: fewer scalar loads per step) vs the tree
bash tools/gpu_steps.sh \
  "r04r_ab|500|REPS=3 bash tools/ab_libs.sh kpr kpr kpr"
