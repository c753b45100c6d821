# Round-3 GPU round AS: int8 GEMV with unsigned-byte widening (sum x * u - 128 sum x)
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny" \
    > gpurun_out/as_tests.log 2>&1 || { tail -40 gpurun_out/as_tests.log; exit 1; }
tail -2 gpurun_out/as_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "int8" \
    > gpurun_out/as_engine.log 2>&1 || { tail -40 gpurun_out/as_engine.log; exit 1; }
tail -2 gpurun_out/as_engine.log
timeout -k 10 600 python -u bench.py --int8 --batch-per-mb 1 --steps 20 --json-out gpurun_out/results/int8_b1_u8.json > gpurun_out/results/int8_b1_u8.log 2>&1 || { tail -20 gpurun_out/results/int8_b1_u8.log; exit 1; }
echo "int8 b1 u8-widening $(python -c "import json;d=json.load(open('gpurun_out/results/int8_b1_u8.json'));print(d['value'], d['ms_per_step'])")"
