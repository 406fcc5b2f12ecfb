#!/bin/bash
# ASan + UBSan over the library's host code on the CPU (no GPU needed): the
# scene builders, cameras, BVH / layer-grid builder, tonemaps and PPM writers,
# driven by tools/host_sanitize.cpp.  The sanitizers instrument host code only
# (-Xarch_host); the driver never launches a kernel.
#   tools/host_sanitize.sh            (exit status 0: clean)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ray-tracing-in-one-weekend_amd
OUT=${TMPDIR:-/tmp}/rtow_host_sanitize
mkdir -p $OUT
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="--offload-arch=gfx950 -std=c++17 -fPIC -g -O1 -fno-omit-frame-pointer -I$ROOT/include -I$PKG/csrc"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC $FLAGS -ffp-contract=off $HSAN -c -o $OUT/rt_kernel.o $PKG/csrc/rt_kernel.hip
$HIPCC $FLAGS $HSAN -c -o $OUT/rt_api.o $PKG/csrc/rt_api.cpp
$HIPCC $FLAGS $HSAN -c -o $OUT/rt_accel.o $PKG/csrc/rt_accel.cpp
$HIPCC $FLAGS $HSAN -c -o $OUT/rt_sched.o $PKG/csrc/rt_sched.hip
$HIPCC $FLAGS $HSAN -x c++ -c -o $OUT/rt_host.o $PKG/csrc/rt_host.cpp
$HIPCC $FLAGS $HSAN -x c++ -c -o $OUT/driver.o $ROOT/tools/host_sanitize.cpp
$HIPCC --offload-arch=gfx950 $HSAN -o $OUT/host_sanitize $OUT/driver.o $OUT/rt_host.o $OUT/rt_kernel.o $OUT/rt_api.o $OUT/rt_accel.o \
  $OUT/rt_sched.o -lpthread
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 $OUT/host_sanitize
