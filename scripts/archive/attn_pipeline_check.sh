#!/bin/bash
# Decode attention with counted vmcnt waits (scalar block-table loads, unconditional clamped K/V
# loads): attention / decode-layer GPU tests, the attention microbench, batch-1 fp8 and the
# default bench.
set -u
mkdir -p gpurun_out/attnpipe
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_layer_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "attn or decode_layer or engine" > gpurun_out/attnpipe/tests.log 2>&1 || { tail -30 gpurun_out/attnpipe/tests.log; exit 1; }
tail -1 gpurun_out/attnpipe/tests.log
timeout -k 10 300 python3 -u scripts/attn_bench.py > gpurun_out/attnpipe/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attnpipe/attn_bench.txt; exit 1; }
grep "{" gpurun_out/attnpipe/attn_bench.txt
timeout -k 10 300 python3 -u scripts/attn_bench.py --cases=1x600 > gpurun_out/attnpipe/attn_b1.txt 2>&1 || { tail -5 gpurun_out/attnpipe/attn_b1.txt; exit 1; }
grep "{" gpurun_out/attnpipe/attn_b1.txt
timeout -k 10 300 python3 -u bench.py --fp8 --batch-per-mb 1 --steps 20 --warmup 3 --json-out gpurun_out/attnpipe/fp8_b1.json > gpurun_out/attnpipe/fp8_b1.log 2>&1 || { tail -20 gpurun_out/attnpipe/fp8_b1.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/attnpipe/fp8_b1.json'));print('fp8 b1', d['value'], d['ms_per_step'])"
timeout -k 10 400 python3 -u bench.py --json-out gpurun_out/attnpipe/bench_default.json > gpurun_out/attnpipe/bench_default.log 2>&1 || { tail -20 gpurun_out/attnpipe/bench_default.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/attnpipe/bench_default.json'));print('default', d['value'], d['ms_per_step'])"
timeout -k 10 400 python3 -u bench.py --fp8 --kv-fp8 --json-out gpurun_out/attnpipe/bench_fp8kv.json > gpurun_out/attnpipe/bench_fp8kv.log 2>&1 || { tail -20 gpurun_out/attnpipe/bench_fp8kv.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/attnpipe/bench_fp8kv.json'));print('fp8+fp8kv', d['value'], d['ms_per_step'])"
