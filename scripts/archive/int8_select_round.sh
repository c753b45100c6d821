#!/bin/bash
# int8 outlier tests, per-kernel probe under rocprofv3, then bench --int8 twice
set -o pipefail
mkdir -p gpurun_out/int8sel
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -k "int8" -x -v --timeout 120 --timeout-method thread > gpurun_out/int8sel/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/int8sel/tests.log; exit 1; }
tail -1 gpurun_out/int8sel/tests.log
rm -rf /tmp/selp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/selp -o run -- python3 scripts/int8_select_probe.py > gpurun_out/int8sel/probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/int8sel/probe.log; exit 1; }
cp "$(find /tmp/selp -name '*kernel_stats.csv' | head -1)" gpurun_out/int8sel/probe_stats.csv
cut -d, -f1-8 gpurun_out/int8sel/probe_stats.csv | head -8
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --int8 --json-out gpurun_out/int8sel/int8_$i.json > gpurun_out/int8sel/int8_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/int8sel/int8_$i.log; exit 1; }
  echo "int8 run $i: $(python -c "import json;d=json.load(open('gpurun_out/int8sel/int8_$i.json'));print(d['value'], d['ms_per_step'])")"
done
