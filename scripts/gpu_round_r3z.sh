# Round-3 GPU round Z: default transport falls back (agreed) from RCCL to the IPC device transport
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multiproc_gpu.py \
    > gpurun_out/z_multiproc.log 2>&1 || { tail -60 gpurun_out/z_multiproc.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/z_multiproc.log | tail -20
