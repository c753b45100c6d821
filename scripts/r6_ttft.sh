# long-context TTFT (Llama-3.1-70B bf16, batch 1) at 32k and 127k prompts + a rocprof breakdown
# of the 32k prefill; engine GPU tests first (the new prefill kernel end to end)
set -u
out=gpurun_out/r6ttft
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $out/engine_tests.log 2>&1 || { tail -30 $out/engine_tests.log; exit 1; }
tail -2 $out/engine_tests.log
for L in 32768 130048; do
  timeout -k 10 400 python -u bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len $L --steps 5 --warmup 2 --json-out $out/ttft_$L.json > $out/ttft_$L.log 2>&1 || { tail -20 $out/ttft_$L.log; exit 1; }
  python -c "import json; d=json.load(open('$out/ttft_$L.json')); print($L, 'prefill_s', d['prefill_s'], 'tok/s', d['value'])"
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof32k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$out/prof32k.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/stats_top.py $(find $out/prof32k -name "*kernel_stats.csv" | head -1) > $out/prof32k_kernel_stats_top.txt && cat $out/prof32k_kernel_stats_top.txt
