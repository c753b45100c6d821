# Same-box A/B of prefill-attention kernel builds (scripts/experiments/build_variant_so.py
# variants): ARMS="base early ..." ; QBS="1 2".  Prints one line per (arm, qb, case).
set -u
ARMS=${ARMS:?ARMS}
QBS=${QBS:-"1 2"}
out=gpurun_out/${TAG:-prefill_ab}
mkdir -p $out
export TMPDIR=/tmp
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" $out/orig.so.keep
rc=0
for arm in $ARMS; do
  if [ "$arm" = base ]; then cp $out/orig.so.keep "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  for qb in $QBS; do
    QB=$qb TAG=$arm-qb$qb timeout -k 10 200 python -u scripts/attn_prefill_bench.py > $out/$arm-qb$qb.txt 2>&1 || { echo "$arm failed"; tail -5 $out/$arm-qb$qb.txt; rc=1; break 2; }
    grep TFLOPs $out/$arm-qb$qb.txt | sed "s/^/$arm /"
  done
done
cp $out/orig.so.keep "$so"
rm -f $out/orig.so.keep
exit $rc
