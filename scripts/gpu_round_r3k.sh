# Round-3 GPU round K: which hipBLASLt kernels serve the small-M decode shapes (stream-K?), then
# the PP=8 IPC rehearsal with every decode GEMM on the tile kernel (DLI_GEMM_LIB=0).
set -u
mkdir -p gpurun_out/prof_blaslt
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_blaslt -o blaslt \
    -- python3 $GRAFT_REPO_ROOT/scripts/blaslt_kernel_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_blaslt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_blaslt.log; exit 1; }
cd $GRAFT_REPO_ROOT
DLI_GEMM_LIB=0 DLI_P2P_TIMEOUT_S=45 DLI_WATCHDOG_S=60 timeout -k 10 600 bash scripts/rehearsal_pp8_ipc.sh
exit $?
