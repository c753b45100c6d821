# Round-3 GPU round T: one-workgroup-per-token RoPE kernel: identity tests, kernel breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k rope \
    > gpurun_out/t_t_rope.log 2>&1 || { tail -30 gpurun_out/t_t_rope.log; exit 1; }
tail -2 gpurun_out/t_t_rope.log
bash scripts/prof_default.sh || exit $?
