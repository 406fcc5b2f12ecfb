#!/bin/bash
# Build a variant of librtow.so with one sed expression applied to the kernel
# source, into build/variants/<name>.so (travels to the box) (A/B experiments only).
#   tools/ab_variant.sh <name> '<sed expression>'
set -e
name=$1; expr=$2
d=build/variants; mkdir -p $d/src_$name
sed "$expr" ray-tracing-in-one-weekend_amd/csrc/rt_render.hip > $d/src_$name/rt_render.hip
if cmp -s $d/src_$name/rt_render.hip ray-tracing-in-one-weekend_amd/csrc/rt_render.hip; then
  echo "variant $name: sed changed nothing" >&2; exit 1
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Iinclude \
  -Iray-tracing-in-one-weekend_amd/csrc -shared -o $d/$name.so $d/src_$name/rt_render.hip \
  ray-tracing-in-one-weekend_amd/csrc/rt_host.cpp
echo "built $d/$name.so"
