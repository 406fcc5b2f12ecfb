bash tools/gpu_steps.sh \
  "r03h_share_c4|300|python tools/rank_share.py --preset c4 --world 8 --rank 0 7 --flags PILOT_SCHEDULE" \
  "r03h_share_c3|300|python tools/rank_share.py --preset c3 --world 8 --rank 0 7 --flags PILOT_SCHEDULE --reps 3" \
  "r03h_c4_trace|400|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r03h_c4kt -o kt -- python3 \$GRAFT_REPO_ROOT/tools/rank_share.py --preset c4 --world 8 --rank 0 --flags PILOT_SCHEDULE" \
  "r03h_image23|300|python -u -m pytest tests/test_reference_gpu.py -k image23 -x -q -s --timeout 200 --timeout-method thread"
