#!/bin/bash
# (run while bench.py, rank_share.py and rank_times.py tuned the grid by default; they now need
#  --grid-tune for that, and --no-grid-tune is gone: the untuned runs are the default)
# rt_tune_grid: its GPU test, the C4 rank-0 share with and without it, the
# headline bench line with it
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k "grid_tune" > gpurun_out/r04tune_test.log 2>&1
timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp 200 --reps 2 --no-grid-tune > gpurun_out/r04tune_c4_200.log 2>&1
timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp 200 --reps 2 >> gpurun_out/r04tune_c4_200.log 2>&1
timeout -k 10 180 python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE > gpurun_out/r04tune_share_c4.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04tune_bench.log 2>&1
echo done
