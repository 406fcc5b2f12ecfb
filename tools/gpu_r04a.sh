# round 4, first GPU call: the sealed opaque-inside rule, 64-bit sums, new tests
bash tools/gpu_steps.sh \
  "r04a_tests|400|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -s" \
  "r04a_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04a_bench|300|python bench.py --steps 20 --warmup 5" \
  "r04a_diff_save|120|RTOW_LIB=build/variants/norule.so python tools/ab_image_diff.py save /tmp/norule.npy" \
  "r04a_diff_rule|120|python tools/ab_image_diff.py diff /tmp/norule.npy" \
  "r04a_diff_r03|120|RTOW_LIB=build/variants/r03.so python tools/ab_image_diff.py diff /tmp/norule.npy" \
  "r04a_ab_libs|300|REPS=4 bash tools/ab_libs.sh norule r03"
