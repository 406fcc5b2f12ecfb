# round 4, final kernel: GPU tests, smoke, C1 bench, every rank's share of the
# headline frame at N = 2, 4, 8 (SCALE expectations), C3 / C4 rank shares at
# their own spp, and the SQ counters of the dielectric-parking variant vs base
bash tools/gpu_steps.sh \
  "r04i_tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "r04i_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04i_bench_c1|200|python bench.py --preset c1 --steps 20 --warmup 5 --no-cpu-baseline" \
  "r04i_rank_times|300|python tools/rank_times.py --pilot --world 2 4 8" \
  "r04i_share_c3|200|python tools/rank_share.py --preset c3 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 2" \
  "r04i_share_c4|300|python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 1" \
  "r04i_pmc_parking|300|bash tools/pmc_ab.sh r04i base xp4"
