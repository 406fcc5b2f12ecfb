bash tools/gpu_steps.sh \
  "r03g_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03g_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03g_bench|300|python bench.py --steps 20 --warmup 5" \
  "r03g_prof|600|bash tools/profile_round.sh r03g --steps 5 --warmup 2" \
  "r03g_shares|600|bash tools/profile_shares.sh r03g 2 4 8" \
  "r03g_c4prof|600|bash tools/c4_profile.sh r03g 100 'c4c c2'"
