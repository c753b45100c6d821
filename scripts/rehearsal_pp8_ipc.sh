# 8-rank PP=8 rehearsal of the DEFAULT bench path on ONE shared GPU: the IPC device transport
# (spinning device waits on the rank's dedicated recv / send / head streams, exactly RCCL's
# stream schedule) with the rotating LM head ON, graphs pre-captured at init, watchdog armed.
# Throughput is not meaningful (8 ranks share one GPU); the protocol and the per-rank record are.
# 32 sequences x 256-token prompts per micro-batch: every one of the 9 x 32 sequences fits the
# 1/8 share of KV each rank gets on the shared GPU, so all of them decode in the timed window.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=ipc DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-120} timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 \
    bench.py --gpus 8 --steps 5 --warmup 2 --batch-per-mb 32 --prompt-len 256 > gpurun_out/rehearsal_pp8_ipc.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp8_ipc.log | tail -1 > gpurun_out/rehearsal_pp8_ipc.json; tail -3 gpurun_out/rehearsal_pp8_ipc.log; exit $rc
