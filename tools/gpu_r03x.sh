bash tools/gpu_steps.sh \
  "r03x_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03x_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03x_ab|400|REPS=3 bash tools/ab_libs.sh preflow" \
  "r03x_share8|200|python tools/rank_share.py --preset c2 --world 8 --rank 0 5 --reps 3 --flags PILOT_SCHEDULE" \
  "r03x_share8_pre|200|RTOW_LIB=build/variants/preflow.so python tools/rank_share.py --preset c2 --world 8 --rank 0 5 --reps 3 --flags PILOT_SCHEDULE" \
  "r03x_bench_c1|120|python bench.py --preset c1 --steps 20 --warmup 3 --no-cpu-baseline"
