bash tools/gpu_steps.sh \
  "r03n_bench_c3|200|python bench.py --preset c3 --steps 3 --warmup 1 --no-cpu-baseline" \
  "r03n_bench_c4|400|python bench.py --preset c4 --steps 1 --warmup 1 --no-cpu-baseline"
