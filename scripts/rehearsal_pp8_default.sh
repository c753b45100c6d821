# 8-rank PP=8 rehearsal of `bench.py --gpus 8` with the DEFAULT transport setting on ONE shared
# GPU: RCCL is tried first (every pair / head communicator), refuses the duplicate device on every
# rank, the ranks agree on the failure and all switch to the IPC device transport (same streams,
# rotating head, watchdog).  Throughput is not meaningful (8 ranks share one GPU).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
unset DLI_TRANSPORT
DLI_SHARE_GPU=1 DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-120} timeout -k 10 700 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29617 \
    bench.py --gpus 8 --steps 5 --warmup 2 --batch-per-mb 32 --prompt-len 256 > gpurun_out/rehearsal_pp8_default.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp8_default.log | tail -1 > gpurun_out/rehearsal_pp8_default.json
grep -E "falling back|RCCL transport unavailable" gpurun_out/rehearsal_pp8_default.log | head -3 | cut -c1-300
tail -2 gpurun_out/rehearsal_pp8_default.log | cut -c1-600; exit $rc
