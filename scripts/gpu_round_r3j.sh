# Round-3 GPU round J: multi-process hardware-queue probe, then the PP=8 IPC rehearsal with the
# finer record (compute_in marks, per-thread waits, recent step shapes).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/hwq_probe_mp.py > gpurun_out/hwq_probe_mp.log 2>&1 || { tail -20 gpurun_out/hwq_probe_mp.log; exit 1; }
grep procs gpurun_out/hwq_probe_mp.log
DLI_P2P_TIMEOUT_S=45 DLI_WATCHDOG_S=60 timeout -k 10 600 bash scripts/rehearsal_pp8_ipc.sh
exit $?
