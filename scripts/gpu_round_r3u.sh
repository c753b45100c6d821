# Round-3 GPU round U: decode attention skips K/V past the sequence end - numerics tests, then the
# decode-step kernel breakdown (bf16, fp8).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernel_canaries_gpu.py \
    > gpurun_out/t_u_kernels.log 2>&1 || { tail -30 gpurun_out/t_u_kernels.log; exit 1; }
tail -2 gpurun_out/t_u_kernels.log
bash scripts/prof_default.sh || exit $?
