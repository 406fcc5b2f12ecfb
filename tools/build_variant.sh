#!/bin/bash
# Build an alternative librtow.so from a modified copy of the render kernel
# (A/B experiments, tools/ab_libs.sh):
#   tools/build_variant.sh <name> <path/to/rt_kernel.hip> [extra hipcc flags]
# -> build/variants/<name>.so, linked with the in-tree rt_api / rt_accel / rt_sched / rt_host objects.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ray-tracing-in-one-weekend_amd
name=$1; src=$2; shift 2
make -s -C "$PKG" build/obj/rt_api.o build/obj/rt_accel.o build/obj/rt_sched.o build/obj/rt_host.o
mkdir -p "$ROOT/build/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
  -I"$PKG/csrc" "$@" -c -o "$ROOT/build/variants/$name.o" "$src"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/build/variants/$name.so" \
  "$ROOT/build/variants/$name.o" "$PKG/build/obj/rt_api.o" "$PKG/build/obj/rt_accel.o" \
  "$PKG/build/obj/rt_sched.o" "$PKG/build/obj/rt_host.o"
echo "build/variants/$name.so"
