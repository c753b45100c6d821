# 8-rank PP=8 rehearsal of the bench path on ONE shared GPU (host transport): checks the 8-process
# protocol end to end with the current kernels; throughput is not meaningful (one GPU, 8 ranks).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=host timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --steps 5 --warmup 2 --batch-per-mb 128 > gpurun_out/rehearsal_pp8.log 2>&1
rc=$?; tail -2 gpurun_out/rehearsal_pp8.log; exit $rc
