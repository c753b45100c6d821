# Round-3 GPU round Y: grouped tile order + non-temporal weight loads in the tile GEMM: GEMM
# numerics tests, then in-step A/B (DLI_GEMM_BNT=1 default vs 0), bf16 and fp8, interleaved.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k "gemm or tile" \
    > gpurun_out/y_tests.log 2>&1 || { tail -30 gpurun_out/y_tests.log; exit 1; }
tail -2 gpurun_out/y_tests.log
for r in 1 0 0 1; do
  DLI_GEMM_BNT=$r timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/y_bnt$r.json > gpurun_out/y_bnt$r.log 2>&1 || { tail -20 gpurun_out/y_bnt$r.log; exit 1; }
  echo "bf16 BNT=$r $(python -c "import json;d=json.load(open('gpurun_out/y_bnt$r.json'));print(d['value'], d['ms_per_step'])")"
done
for r in 1 0; do
  DLI_GEMM_BNT=$r timeout -k 10 300 python -u bench.py --fp8 --kv-fp8 --steps 10 --warmup 3 --json-out gpurun_out/y_fp8_bnt$r.json > gpurun_out/y_fp8_bnt$r.log 2>&1 || { tail -20 gpurun_out/y_fp8_bnt$r.log; exit 1; }
  echo "fp8+fp8kv BNT=$r $(python -c "import json;d=json.load(open('gpurun_out/y_fp8_bnt$r.json'));print(d['value'], d['ms_per_step'])")"
done
