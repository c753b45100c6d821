# 8-rank PP=8 rehearsal over STRICT RCCL on ONE shared GPU: each rank claims a host of its own
# (DLI_RCCL_RANK_HOSTS=1 -> NCCL_HOSTID), so RCCL accepts the ranks that share the card and
# connects every stage pair and head pair through its socket transport on loopback (not xGMI: the
# bytes cross host memory).  Same config as rehearsal_pp8_rows512.sh (Llama-3-70B width, 16
# layers, 8 ranks x 9 micro-batches x 512 rows, rotating head, fp8 KV, graphs, watchdog), hop
# digests on (bench.py's default).  Throughput is not meaningful; the RCCL protocol, the
# communicators on the transport's streams and the hop integrity record are what is checked.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=rccl DLI_RCCL_RANK_HOSTS=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT \
  DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-240} timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29641 \
    bench.py --gpus 8 --steps ${STEPS:-5} --warmup 2 --num-layers 16 --batch-per-mb 512 --prompt-len 512 \
    --kv-fp8 --max-batched-tokens 4096 > gpurun_out/rehearsal_pp8_rccl.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp8_rccl.log | tail -1 > gpurun_out/rehearsal_pp8_rccl.json
grep -c "via NET/Socket" gpurun_out/rehearsal_pp8_rccl.log
tail -3 gpurun_out/rehearsal_pp8_rccl.log | cut -c1-600; exit $rc
