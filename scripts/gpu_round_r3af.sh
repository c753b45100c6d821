# Round-3 GPU round AF: register-resident top-k / top-p sampler - numerics tests + timing vs radix
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k sample \
    > gpurun_out/af_tests.log 2>&1 || { tail -40 gpurun_out/af_tests.log; exit 1; }
tail -2 gpurun_out/af_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "sampl or seed or rotat" \
    > gpurun_out/af_engine.log 2>&1 || { tail -40 gpurun_out/af_engine.log; exit 1; }
tail -2 gpurun_out/af_engine.log
timeout -k 10 300 python -u scripts/sample_probe.py > gpurun_out/af_sample.log 2>&1 || { tail -30 gpurun_out/af_sample.log; exit 1; }
cat gpurun_out/af_sample.log
