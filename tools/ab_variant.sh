#!/bin/bash
# Build a variant of librtow.so with one sed expression applied to the kernel
# source, into build/variants/<name>.so (travels to the box) (A/B experiments only).
#   tools/ab_variant.sh <name> '<sed expression>'
set -e
name=$1; expr=$2
d=build/variants; mkdir -p $d/src_$name
sed "$expr" ray-tracing-in-one-weekend_amd/csrc/rt_kernel.hip > $d/src_$name/rt_kernel.hip
if cmp -s $d/src_$name/rt_kernel.hip ray-tracing-in-one-weekend_amd/csrc/rt_kernel.hip; then
  echo "variant $name: sed changed nothing" >&2; exit 1
fi
tools/build_variant.sh $name $d/src_$name/rt_kernel.hip > /dev/null
echo "built $d/$name.so"
