set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sk in 0 1; do
  rm -rf /tmp/prof_sk$sk
  DLI_TILE_SK=$sk timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_sk$sk -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_sk$sk.log 2>&1 || exit $?
  f=$(find /tmp/prof_sk$sk -name "*kernel_trace.csv" | head -1)
  python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_sk${sk}_breakdown.txt || exit $?
  head -8 gpurun_out/prof_sk${sk}_breakdown.txt
done
