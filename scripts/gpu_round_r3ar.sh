# Round-3 GPU round AR: int8-weight GEMV for 1-2 row decode (LLM.int8 mode) - numerics, engine
# int8 tests, batch-1 bench with the GEMV vs the LLM.int8 tile path
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny" \
    > gpurun_out/ar_tests.log 2>&1 || { tail -40 gpurun_out/ar_tests.log; exit 1; }
tail -2 gpurun_out/ar_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_gemm_gpu.py -k "int8" \
    > gpurun_out/ar_engine.log 2>&1 || { tail -40 gpurun_out/ar_engine.log; exit 1; }
tail -2 gpurun_out/ar_engine.log
for g in 1 0; do
  DLI_INT8_GEMV=$g timeout -k 10 600 python -u bench.py --int8 --batch-per-mb 1 --steps 20 --json-out gpurun_out/results/int8_b1_gemv$g.json > gpurun_out/results/int8_b1_gemv$g.log 2>&1 || { tail -20 gpurun_out/results/int8_b1_gemv$g.log; exit 1; }
  echo "int8 b1 GEMV=$g $(python -c "import json;d=json.load(open('gpurun_out/results/int8_b1_gemv$g.json'));print(d['value'], d['ms_per_step'])")"
done
