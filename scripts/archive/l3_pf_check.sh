#!/bin/bash
# Infinity-Cache warm-up of the O GEMV's weights during batch-1 attention: numerics test, the
# standalone probe (cold vs warm GEMV), then fp8 / bf16 batch-1 benches with and without it.
set -u
mkdir -p gpurun_out/l3pf
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "l3_prefetch or attn_decode" > gpurun_out/l3pf/tests.log 2>&1 || { tail -30 gpurun_out/l3pf/tests.log; exit 1; }
tail -1 gpurun_out/l3pf/tests.log
timeout -k 10 200 python3 -u scripts/l3_prefetch_probe.py fp8 > gpurun_out/l3pf/probe_fp8.txt 2>&1 || { tail -5 gpurun_out/l3pf/probe_fp8.txt; exit 1; }
cat gpurun_out/l3pf/probe_fp8.txt
timeout -k 10 200 python3 -u scripts/l3_prefetch_probe.py bf16 > gpurun_out/l3pf/probe_bf16.txt 2>&1 || { tail -5 gpurun_out/l3pf/probe_bf16.txt; exit 1; }
cat gpurun_out/l3pf/probe_bf16.txt
run() {  # name, extra env..., bench flag
  local name=$1; shift
  local flag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py $flag --batch-per-mb 1 --steps 20 --warmup 3 --json-out gpurun_out/l3pf/$name.json > gpurun_out/l3pf/$name.log 2>&1 || { tail -20 gpurun_out/l3pf/$name.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/l3pf/$name.json'));print('$name', d['value'], 'tok/s', d['ms_per_step'], 'ms')"
}
run fp8_off --fp8 DLI_L3_PF=0 && run fp8_on --fp8 DLI_L3_PF=1 && run fp8_on_s06 --fp8 DLI_L3_PF=1 DLI_L3_PF_SPLIT=0.6 && run fp8_off2 --fp8 DLI_L3_PF=0 && run fp8_on2 --fp8 DLI_L3_PF=1 && run bf16_off "" DLI_L3_PF=0 && run bf16_on "" DLI_L3_PF=1
