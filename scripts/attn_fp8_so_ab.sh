# fp8-KV decode attention probe (scripts/attn_fp8kv_probe.py) on extension variants, interleaved
set -u
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" /tmp/base.so
rc=0
for arm in ${ARMS:-base fp8one base fp8one}; do
  if [ $arm = base ]; then cp /tmp/base.so "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  echo "== $arm"
  timeout -k 10 300 python -u scripts/attn_fp8kv_probe.py ${CASES:+--cases=$CASES} 2>&1 | grep '"B"' || { rc=1; break; }
done
cp /tmp/base.so "$so"
exit $rc
