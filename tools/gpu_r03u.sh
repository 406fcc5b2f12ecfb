bash tools/gpu_steps.sh \
  "r03u_bench|300|python bench.py --steps 20 --warmup 5" \
  "r03u_bench_c1|120|python bench.py --preset c1 --steps 20 --warmup 3"
