# Round-3 GPU round L: PP=8 IPC rehearsal with the defaults (shared GPU => no library GEMMs),
# then the whole GPU test suite.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_P2P_TIMEOUT_S=45 DLI_WATCHDOG_S=60 timeout -k 10 420 bash scripts/rehearsal_pp8_ipc.sh || exit $?
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/t_l_all.log 2>&1 || { tail -30 gpurun_out/t_l_all.log; exit 1; }
tail -3 gpurun_out/t_l_all.log
