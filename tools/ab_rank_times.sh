#!/bin/bash
# Per-rank share times (tools/rank_times.py --pilot) for alternative librtow
# builds, base first and last (GPU box):  tools/ab_rank_times.sh <variant> ...
set -e
run() {
  local lib=ray-tracing-in-one-weekend_amd/librtow.so
  [ "$1" != base ] && lib=build/variants/$1.so
  RTOW_LIB=$lib timeout -k 10 120 python tools/rank_times.py --world ${WORLDS:-8} --pilot | sed "s/^/$1 /"
}
run base
for v in "$@"; do run $v; done
run base
