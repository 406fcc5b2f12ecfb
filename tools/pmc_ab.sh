#!/bin/bash
# SQ counters of one headline frame per librtow build (GPU box):
#   tools/pmc_ab.sh <tag> <variant|base> ...   -> gpurun_out/pmcab_<tag>/<variant>/
# (base = the in-tree build; others build/variants/<name>.so)
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  out=$GRAFT_REPO_ROOT/gpurun_out/pmcab_$tag/$v
  mkdir -p $out
  lib=$GRAFT_REPO_ROOT/ray-tracing-in-one-weekend_amd/librtow.so
  [ "$v" != base ] && lib=$GRAFT_REPO_ROOT/build/variants/$v.so
  export RTOW_LIB=$lib
  timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY} \
    --output-format csv -d $out -o p -- python3 $GRAFT_REPO_ROOT/tools/ab_flags.py --reps 1 ${AB_FLAGS:-ACCEL_BVH+PILOT_SCHEDULE} > $out/run.log 2>&1
  python3 - "$out" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
f = glob.glob(out + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f)):
    if os.environ.get("KERNEL", "render_kernel<false, false, true, false, true, 1, false>") in row["Kernel_Name"]:
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
print(out.split("/")[-1], {k: f"{v:.4g}" for k, v in sorted(acc.items())})
PY
done
