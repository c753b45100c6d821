#!/bin/bash
# rocprofv3 decode breakdown of bench.py --fp8 (MX down projection) and --fp8 --kv-fp8
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in fp8 fp8kv; do
  extra="--fp8"; [ $cfg = fp8kv ] && extra="--fp8 --kv-fp8"
  rm -rf /tmp/prof_$cfg
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$cfg -o run -- python3 bench.py --steps 5 --warmup 2 $extra --json-out gpurun_out/prof_${cfg}_bench.json > gpurun_out/prof_$cfg.log 2>&1 || exit $?
  f=$(find /tmp/prof_$cfg -name "*kernel_trace.csv" | head -1)
  s=$(find /tmp/prof_$cfg -name "*kernel_stats.csv" | head -1)
  cp "$s" gpurun_out/prof_${cfg}_kernel_stats.csv
  python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_${cfg}_breakdown.txt || exit $?
  head -14 gpurun_out/prof_${cfg}_breakdown.txt
done
