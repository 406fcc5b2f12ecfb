# round 4, final kernel with rt_tune_grid: the GPU suite and smoke
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'"
