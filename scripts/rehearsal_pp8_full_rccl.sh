# `bench.py --gpus 8` with the FULL Llama-3-70B (80 layers, 10 per rank) over STRICT RCCL on ONE
# shared GPU (DLI_RCCL_RANK_HOSTS=1: per-rank RCCL hosts, loopback sockets): every pair and head
# communicator, rotating head, graphs, hop digests.  32 x 256-token sequences per micro-batch so
# the 1/8 KV share per rank holds them all.  Throughput is not meaningful.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=rccl DLI_RCCL_RANK_HOSTS=1 DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-240} \
  timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29644 \
    bench.py --gpus 8 --steps 5 --warmup 2 --batch-per-mb 32 --prompt-len 256 > gpurun_out/rehearsal_pp8_full_rccl.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp8_full_rccl.log | tail -1 > gpurun_out/rehearsal_pp8_full_rccl.json
grep -v NCCL gpurun_out/rehearsal_pp8_full_rccl.log | tail -2 | cut -c1-400; exit $rc
