#!/bin/bash
# The one runner of every GPU session (round 5: the per-session scripts of
# rounds 3-4 are gone).  Runs GPU steps in order, each under its own time
# limit.  A step that fails normally (exit 1: a test failure) does not stop
# the sequence; a crash, abort, fault or time-out (anything else non-zero), or
# a GPU fault the runtime prints in the step's log, ends it -- nothing more
# touches the GPU after that.
#   tools/gpu_steps.sh "name|seconds|command" ...
# The argument list is written to gpurun_out/<first step>.steps, which is
# committed under profiles/ with the logs it produced.
mkdir -p gpurun_out
first="${1%%|*}"
printf '%s\n' "$@" > "gpurun_out/$first.steps"
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
  # a device fault the runtime reported (the process may still exit 0 or 1):
  # nothing more touches the GPU
  if grep -qE "HSA_STATUS_ERROR|Memory access fault|MEMORY_APERTURE_VIOLATION" "gpurun_out/$name.log"; then
    echo "== stopping: $name reported a GPU fault"
    exit 3
  fi
done
