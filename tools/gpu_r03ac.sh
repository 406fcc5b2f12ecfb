bash tools/gpu_steps.sh \
  "r03ac_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03ac_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r03ac_bench|300|python bench.py --steps 20 --warmup 5"
