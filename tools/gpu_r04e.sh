# round 4: GPU tests on the tree (compacted extras + lens branch + folded face flip + no splats),
# A/B of the shading-record hoist (xi) and two walk-setup micro changes (xj)
bash tools/gpu_steps.sh \
  "r04e_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r04e_ab|500|REPS=3 bash tools/ab_libs.sh xi xj"
