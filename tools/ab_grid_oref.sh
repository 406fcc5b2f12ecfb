set -e
r() { RTOW_LIB=$1 timeout -k 10 90 python tools/ab_flags.py --reps 2 ACCEL_BVH+PILOT_SCHEDULE | sed "s/^/$2 /"; }
r ray-tracing-in-one-weekend_amd/librtow.so base
for o in 12 16 24 32 48; do RTOW_GRID_OREF=$o r build/variants/vG.so oref$o; done
r ray-tracing-in-one-weekend_amd/librtow.so base
