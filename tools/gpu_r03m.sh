bash tools/gpu_steps.sh \
  "r03m_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03m_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03m_bench|300|python bench.py --steps 20 --warmup 5" \
  "r03m_prof|600|bash tools/profile_round.sh r03m --steps 5 --warmup 2"
