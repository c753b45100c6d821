# Round-3 GPU round H: entry/passed progress words + frozen releases after a failure, per-stream
# device marks; the IPC transport tests, then the PP=8 IPC rehearsal (diagnostic record).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_streams_gpu.py tests/test_multiproc_gpu.py > gpurun_out/t_h_streams.log 2>&1 || { tail -30 gpurun_out/t_h_streams.log; exit 1; }
tail -2 gpurun_out/t_h_streams.log
DLI_P2P_TIMEOUT_S=45 DLI_WATCHDOG_S=60 timeout -k 10 600 bash scripts/rehearsal_pp8_ipc.sh
exit $?
