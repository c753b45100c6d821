# Round-3 GPU round AT: last check of the committed tree's build - GEMV / sampler / GEMM tests + smoke
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py \
    > gpurun_out/at_tests.log 2>&1 || { tail -40 gpurun_out/at_tests.log; exit 1; }
tail -2 gpurun_out/at_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/at_smoke.log 2>&1 || { tail -5 gpurun_out/at_smoke.log; exit 1; }
tail -1 gpurun_out/at_smoke.log
