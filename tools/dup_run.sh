set -e
mkdir -p gpurun_out
timeout -k 10 60 python tools/ab_flags.py --reps 2 ACCEL_BVH > gpurun_out/dup_base.log 2>&1
for v in box extras rootsqrt pcg sincos refine camera; do
  RTOW_LIB=build/variants/dup_$v.so timeout -k 10 60 python tools/ab_flags.py --reps 2 ACCEL_BVH > gpurun_out/dup_$v.log 2>&1
done
timeout -k 10 60 python tools/ab_flags.py --reps 2 ACCEL_BVH > gpurun_out/dup_base2.log 2>&1
timeout -k 10 120 python tools/work_profile.py > gpurun_out/work.log 2>&1
bash tools/stall_profile.sh r01c
grep -h kernel_ms gpurun_out/dup_*.log
