set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_i8
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_i8 -o run -- python3 bench.py --int8 --steps 3 --warmup 1 > gpurun_out/prof_int8.log 2>&1 || exit $?
f=$(find /tmp/prof_i8 -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py "$f" --steps 2 > gpurun_out/prof_int8_breakdown.txt || exit $?
head -24 gpurun_out/prof_int8_breakdown.txt
