# (run while bench.py, rank_share.py and rank_times.py tuned the grid by default; they now need
#  --grid-tune for that, and --no-grid-tune is gone: the untuned runs are the default)
# round 4, final kernel with rt_tune_grid: GPU tests, smoke, bench, rocprofv3 kernel trace + PMC
# passes of the headline frame and the 1/2, 1/4, 1/8 shares, C1, every rank's
# share at N = 2, 4, 8, C3 / C4 rank shares at their own spp
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py --steps 20 --warmup 5" \
  "prof|600|bash tools/profile_round.sh r04zt" \
  "shares|600|bash tools/profile_shares.sh r04zt 2 4 8" \
  "bench_c1|200|python bench.py --preset c1 --steps 20 --warmup 5 --no-cpu-baseline" \
  "rank_times|300|python tools/rank_times.py --pilot --world 2 4 8" \
  "share_c3|200|python tools/rank_share.py --preset c3 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 2" \
  "share_c4|300|python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 1"
