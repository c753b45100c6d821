# Round-3 GPU round AK: sampler register path vs radix path (identical tokens)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sample" \
    > gpurun_out/ak_tests.log 2>&1 || { tail -40 gpurun_out/ak_tests.log; exit 1; }
tail -2 gpurun_out/ak_tests.log
