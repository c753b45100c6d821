# start-up warm-up of the hipBLASLt prefill projections: first-request TTFT with and without,
# alternating, same box (+ engine GPU tests)
set -u
out=gpurun_out/r6warm
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $out/engine_tests.log 2>&1 || { tail -30 $out/engine_tests.log; exit 1; }
tail -1 $out/engine_tests.log
for i in 1 2; do
  for w in 1 0; do
    DLI_KERNELS=warm_library_gemms=$w timeout -k 10 600 python -u bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 2 --warmup 1 --json-out $out/w${w}_$i.json > $out/w${w}_$i.log 2>&1 || { tail -20 $out/w${w}_$i.log; exit 1; }
    python -c "import json; d=json.load(open('$out/w${w}_$i.json')); print('warm=$w run $i prefill_s', d['prefill_s'], 'init_s', d['init_s'])"
  done
done
