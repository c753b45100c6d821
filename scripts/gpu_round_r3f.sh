# Round-3 GPU round F: does a host->device copy queued behind a spinning wait on one stream hold
# up other streams' copies (shared copy-engine queue)?  With SDMA (default) and without; then the
# IPC PP=8 rehearsal with copy kernels (+ device progress words in the abort record).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/queue_probe.py --copies-only --out gpurun_out/copies_sdma_on.json \
    > gpurun_out/copies_sdma_on.log 2>&1 || exit $?
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u scripts/queue_probe.py --copies-only \
    --out gpurun_out/copies_sdma_off.json > gpurun_out/copies_sdma_off.log 2>&1 || exit $?
cat gpurun_out/copies_sdma_on.log gpurun_out/copies_sdma_off.log | grep isolated
DLI_P2P_TIMEOUT_S=60 bash scripts/rehearsal_pp8_ipc.sh
exit $?
