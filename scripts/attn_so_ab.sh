set -u
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" /tmp/base.so
rc=0
for arm in base sb4 sb5 base sb4 sb5; do
  if [ $arm = base ]; then cp /tmp/base.so "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  echo "== $arm"
  timeout -k 10 200 python -u scripts/attn_bench.py --cases=512x600,512x1100,64x4096,16x8192 2>&1 | grep "'B'" || { rc=1; break; }
done
cp /tmp/base.so "$so"
exit $rc
