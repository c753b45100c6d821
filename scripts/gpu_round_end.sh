#!/bin/bash
# Round-end evidence on one MI355X, in one call: every GPU test, smoke(), the default bench, then a
# rocprofv3 per-kernel decode breakdown of bench.py for bf16, fp8 and fp8 + fp8 KV.  Every step has
# its own time limit and the first failure ends the script.
set -u
out=gpurun_out/round_end
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests_all.log 2>&1 || { tail -30 $out/gpu_tests_all.log; exit 1; }
tail -2 $out/gpu_tests_all.log
timeout -k 10 300 python3 -u __graft_entry__.py smoke > $out/smoke.log 2>&1 \
  || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python3 -u bench.py > $out/bench_default.json 2> $out/bench_default.err \
  || { tail -20 $out/bench_default.err; exit 1; }
tail -1 $out/bench_default.json
for cfg in bf16 fp8 fp8kv; do
  extra=""
  [ $cfg = fp8 ] && extra="--fp8"
  [ $cfg = fp8kv ] && extra="--fp8 --kv-fp8"
  rm -rf /tmp/prof_$cfg
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$cfg -o run \
    -- python3 bench.py --steps 5 --warmup 2 $extra --json-out $out/prof_${cfg}_bench.json \
    > $out/prof_$cfg.log 2>&1 || { tail -20 $out/prof_$cfg.log; exit 1; }
  f=$(ls /tmp/prof_$cfg/*/*kernel_trace.csv /tmp/prof_$cfg/*kernel_trace.csv 2>/dev/null | sed -n 1p)
  s=$(ls /tmp/prof_$cfg/*/*kernel_stats.csv /tmp/prof_$cfg/*kernel_stats.csv 2>/dev/null | sed -n 1p)
  cp "$s" $out/prof_${cfg}_kernel_stats.csv
  python3 scripts/analyze_trace.py "$f" --steps 3 > $out/prof_${cfg}_breakdown.txt || exit 1
  sed -n 1,12p $out/prof_${cfg}_breakdown.txt
done
