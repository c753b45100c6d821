# DP x PP over STRICT RCCL on ONE shared GPU: 4 ranks = 2 pipeline replicas x 2 stages, each
# replica with its own RCCL pair / head communicators (DLI_RCCL_RANK_HOSTS=1: loopback sockets).
# Llama-3-70B width, 16 layers, 512-row micro-batches, hop digests on.  Throughput not meaningful.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=rccl DLI_RCCL_RANK_HOSTS=1 DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-240} \
  timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29643 \
    bench.py --gpus 4 --dp 2 --steps ${STEPS:-5} --warmup 2 --num-layers 16 --batch-per-mb 512 \
    --prompt-len 512 --kv-fp8 --max-batched-tokens 4096 > gpurun_out/rehearsal_dp2pp2_rccl.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_dp2pp2_rccl.log | tail -1 > gpurun_out/rehearsal_dp2pp2_rccl.json
grep -v "NCCL" gpurun_out/rehearsal_dp2pp2_rccl.log | tail -3 | cut -c1-400; exit $rc
