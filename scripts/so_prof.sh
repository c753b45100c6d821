# rocprofv3 decode breakdowns of kernel-extension variants on one box (see so_ab.sh):
# ARMS="base hpw16" TAG=name bash scripts/so_prof.sh [bench args]
set -u
TAG=${TAG:-so_prof}
ARMS=${ARMS:?ARMS}
out=gpurun_out/$TAG
mkdir -p $out
export TMPDIR=/tmp
so=$(ls distributed_llm_inference/_C*.so)
cp "$so" /tmp/orig_so.keep
rc=0
for arm in $ARMS; do
  if [ "$arm" = base ]; then cp /tmp/orig_so.keep "$so"; else cp tools_bin/variants/$arm/$(basename "$so") "$so"; fi
  rm -rf /tmp/prof_$arm
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$arm -o run -- python3 bench.py --steps 5 --warmup 2 "$@" > $out/$arm.log 2>&1 || { rc=$?; break; }
  f=$(find /tmp/prof_$arm -name "*kernel_trace.csv" | head -1)
  python3 scripts/analyze_trace.py "$f" --steps 3 > $out/$arm.breakdown.txt || { rc=$?; break; }
  echo "== $arm"; head -12 $out/$arm.breakdown.txt
done
cp /tmp/orig_so.keep "$so"
exit $rc
