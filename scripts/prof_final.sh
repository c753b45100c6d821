set -u
out=gpurun_out/prof_final
mkdir -p $out
export TMPDIR=/tmp
for cfg in bf16 fp8kv; do
  extra=""; [ $cfg = fp8kv ] && extra="--fp8 --kv-fp8"
  rm -rf /tmp/prof_$cfg
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$cfg -o run -- python3 bench.py --steps 5 --warmup 2 $extra --json-out $out/prof_${cfg}_bench.json > $out/prof_$cfg.log 2>&1 || exit 1
  f=$(ls /tmp/prof_$cfg/*/*kernel_trace.csv /tmp/prof_$cfg/*kernel_trace.csv 2>/dev/null | sed -n 1p)
  python3 scripts/analyze_trace.py "$f" --steps 3 > $out/prof_${cfg}_breakdown.txt || exit 1
  sed -n 1,12p $out/prof_${cfg}_breakdown.txt
done
