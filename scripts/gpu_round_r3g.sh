# Round-3 GPU round G: per-step host<->device transfers as copy kernels over device-mapped host
# memory (executor staging, token ring).  Copy-coupling probe (memcpy vs copy kernel), streams +
# multi-process tests, the whole GPU suite, the PP=8 IPC rehearsal, the default 1-GPU bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u scripts/queue_probe.py --copies-only --out gpurun_out/copies_g.json \
    > gpurun_out/copies_g.log 2>&1 || exit $?
grep -o '"isolated": [a-z]*' gpurun_out/copies_g.json
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_streams_gpu.py tests/test_multiproc_gpu.py > gpurun_out/t_g_streams.log 2>&1 || { tail -30 gpurun_out/t_g_streams.log; exit 1; }
tail -3 gpurun_out/t_g_streams.log
DLI_P2P_TIMEOUT_S=60 timeout -k 10 600 bash scripts/rehearsal_pp8_ipc.sh || exit $?
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_g.log 2>&1 || { tail -20 gpurun_out/bench_g.log; exit 1; }
grep metric gpurun_out/bench_g.log
