#!/bin/bash
# Full validation on one GPU: every GPU test, smoke, then the default bench and the fp8 variants.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 600 python bench.py --json-out gpurun_out/v_bf16.json > gpurun_out/v_bf16.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --fp8 --json-out gpurun_out/v_fp8.json > gpurun_out/v_fp8.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --fp8 --kv-fp8 --json-out gpurun_out/v_fp8kv.json > gpurun_out/v_fp8kv.log 2>&1 || exit $?
python -c "
import json
for f in ('v_bf16', 'v_fp8', 'v_fp8kv'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, d['value'], d['ms_per_step'])"
