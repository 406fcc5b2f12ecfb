bash tools/gpu_steps.sh \
  "r03p_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03p_bench_c4|400|python bench.py --preset c4 --steps 1 --warmup 1 --no-cpu-baseline" \
  "r03p_share_c4|200|python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE" \
  "r03p_bench_c3|200|python bench.py --preset c3 --steps 3 --warmup 1 --no-cpu-baseline" \
  "r03p_bench|300|python bench.py --steps 20 --warmup 5" \
  "r03p_prof|600|bash tools/profile_round.sh r03p --steps 5 --warmup 2"
