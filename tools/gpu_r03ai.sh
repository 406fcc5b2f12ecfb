bash tools/gpu_steps.sh \
  "r03ai_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03ai_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03ai_bench|300|python bench.py --steps 20 --warmup 5"
