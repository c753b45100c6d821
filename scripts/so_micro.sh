# Same-box A/B of kernel-extension builds on a microbenchmark (see so_ab.sh for the bench.py
# form): each arm's _C is copied over the in-tree one, then the command runs.
# Usage: ARMS="base t64 base t64" bash scripts/so_micro.sh python scripts/rope_bench.py --kv-fp8
set -u
ARMS=${ARMS:?ARMS: base and variant names}
export TMPDIR=/tmp
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" /tmp/so_micro_orig.keep
rc=0
for arm in $ARMS; do
  if [ "$arm" = base ]; then cp /tmp/so_micro_orig.keep "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  echo "== $arm"
  timeout -k 10 120 "$@" || { rc=$?; echo "failed: $arm rc=$rc"; break; }
done
cp /tmp/so_micro_orig.keep "$so"
exit $rc
