# 2-rank PP=2 rehearsal of the driver's N=2 bench call on ONE shared GPU: the full Llama-3-70B
# (40 layers per rank), 512 sequences per micro-batch, IPC device transport (RCCL cannot pair two
# ranks on one GPU).  Throughput is meaningless (both ranks share the GPU); this checks that the
# N=2 command line runs end to end and prints its JSON line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=ipc DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-300} timeout -k 10 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 \
    bench.py --gpus 2 --steps ${STEPS:-10} --warmup 3 > gpurun_out/rehearsal_pp2_full.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp2_full.log | tail -1 > gpurun_out/rehearsal_pp2_full.json
tail -3 gpurun_out/rehearsal_pp2_full.log | cut -c1-400; exit $rc
