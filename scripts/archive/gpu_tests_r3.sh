# Round-3 GPU validation: the new stream / IPC / rotating-head tests first, then the whole GPU suite.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_streams_gpu.py tests/test_multiproc_gpu.py > gpurun_out/t_streams_mp.log 2>&1
rc=$?; tail -3 gpurun_out/t_streams_mp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    --deselect tests/test_multiproc_gpu.py --deselect tests/test_streams_gpu.py > gpurun_out/t_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu_all.log; exit $rc
