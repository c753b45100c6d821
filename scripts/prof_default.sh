# rocprofv3 kernel trace of the default bench (bf16) and the fp8 variant; per-kernel decode-step breakdown
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in bf16 fp8; do
  extra=""; [ $cfg = fp8 ] && extra="--fp8"
  rm -rf /tmp/prof_$cfg
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$cfg -o run -- python3 bench.py --steps 5 --warmup 2 $extra --json-out gpurun_out/prof_${cfg}_bench.json > gpurun_out/prof_$cfg.log 2>&1 || exit $?
  f=$(find /tmp/prof_$cfg -name "*kernel_trace.csv" | head -1)
  s=$(find /tmp/prof_$cfg -name "*kernel_stats.csv" | head -1)
  cp "$s" gpurun_out/prof_${cfg}_kernel_stats.csv
  cyc="~gemm4_kernel<4,:3"; [ $cfg = fp8 ] && cyc="dli::gemm_tile_kernel<4, 3, false, 1>:2"
  python3 scripts/analyze_trace.py "$f" --steps 3 --cycle "$cyc" > gpurun_out/prof_${cfg}_breakdown.txt || exit $?
  cat gpurun_out/prof_${cfg}_breakdown.txt
done
