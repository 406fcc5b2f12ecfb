#!/bin/bash
# Run GPU steps in order, each under its own time limit.  A step that fails
# normally (exit 1: a test failure) does not stop the sequence; a crash,
# abort, fault or time-out (anything else non-zero) ends it -- nothing more
# touches the GPU after that.
#   tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name exit $rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: $name ended with $rc"
    exit $rc
  fi
done
