# Same-box A/B of kernel-extension builds: ARMS lists "base" (the in-tree _C) and variant names
# built by scripts/experiments/build_variant_so.py (tools_bin/variants/<name>/); each arm's .so is
# copied over the in-tree one before its bench run, the original is restored at the end.
# Usage: TAG=name ARMS="base depth3 base depth3" bash scripts/so_ab.sh [bench args]
set -u
TAG=${TAG:-so_ab}
ARMS=${ARMS:?ARMS: base and variant names}
out=gpurun_out/$TAG
mkdir -p $out
export TMPDIR=/tmp
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" $out/orig.so.keep
n=0
rc=0
for arm in $ARMS; do
  n=$((n + 1))
  if [ "$arm" = base ]; then cp $out/orig.so.keep "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  log=$out/$n-$arm.log
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > "$log" 2>&1 || { echo "bench $arm failed"; tail -20 "$log"; rc=1; break; }
  grep '^{' "$log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])"
done
cp $out/orig.so.keep "$so"
rm -f $out/orig.so.keep
exit $rc
