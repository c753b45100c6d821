# The driver's N=2 bench call (full Llama-3-70B, 40 layers per rank, default micro-batching) on
# ONE shared GPU over STRICT RCCL: DLI_RCCL_RANK_HOSTS=1 gives each rank its own RCCL host, so the
# pair communicator forms (loopback sockets, not xGMI).  Checks the full-size command line end to
# end on RcclTransport with the hop digests on; throughput is not meaningful.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=rccl DLI_RCCL_RANK_HOSTS=1 DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-300} \
  timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29642 \
    bench.py --gpus 2 --steps ${STEPS:-10} --warmup 3 > gpurun_out/rehearsal_pp2_full_rccl.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp2_full_rccl.log | tail -1 > gpurun_out/rehearsal_pp2_full_rccl.json
tail -3 gpurun_out/rehearsal_pp2_full_rccl.log | cut -c1-400; exit $rc
