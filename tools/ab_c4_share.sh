for v in base fSLP base fSLP; do
  lib=ray-tracing-in-one-weekend_amd/librtow.so; [ $v != base ] && lib=build/variants/$v.so
  echo "$v $(RTOW_LIB=$lib timeout -k 10 120 python tools/rank_share.py --preset c4 --world 8 --rank 0 --spp 200 2>/dev/null | tail -1 | cut -c1-200)"
done
