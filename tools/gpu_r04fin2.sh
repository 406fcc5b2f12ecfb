# round 4, final: tuner with three pilot passes -- GPU suite, smoke, three
# bench runs (the tuner's pick and its spread), the profile of the bench
bash tools/gpu_steps.sh \
  "tests|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py --steps 20 --warmup 5" \
  "bench2|300|python bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
  "bench3|300|python bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
  "prof|600|bash tools/profile_round.sh r04zu" \
  "share_c4|300|python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 1"
