# round 4, final kernel: bench, rocprofv3 kernel trace + PMC passes of the
# headline frame and of the 1/2, 1/4, 1/8 rank shares
bash tools/gpu_steps.sh \
  "bench|300|python bench.py --steps 20 --warmup 5" \
  "prof|700|bash tools/profile_round.sh r04h" \
  "shares|700|bash tools/profile_shares.sh r04h 2 4 8"
