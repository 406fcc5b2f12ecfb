# round 4, last check of the tree the driver runs: GPU suite, smoke, default bench
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py"
