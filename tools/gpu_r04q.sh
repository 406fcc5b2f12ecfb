# round 4: GPU tests, smoke and bench on the tree (material blocks, extras pointers,
# divergent main loop, row table with valid-column counts), C4 share at 200 spp
bash tools/gpu_steps.sh \
  "r04q_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r04q_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04q_bench|300|python bench.py --steps 20 --warmup 5" \
  "r04q_c4|200|python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp 200 --reps 2 --flags PILOT_SCHEDULE"
