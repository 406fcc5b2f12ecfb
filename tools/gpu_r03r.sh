bash tools/gpu_steps.sh \
  "r03r_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03r_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03r_ab|400|REPS=3 bash tools/ab_libs.sh prepersist" \
  "r03r_bench_c1|120|python bench.py --preset c1 --steps 20 --warmup 3 --no-cpu-baseline"
