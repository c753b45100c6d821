# PP=2 and PP=4 rehearsals of `bench.py --gpus N` with the DEFAULT transport setting on ONE shared
# GPU (the driver's N=2 / N=4 scaling runs, minus real RCCL: refused on the shared GPU, agreed IPC
# fallback).  Throughput is not meaningful (ranks share one GPU).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
unset DLI_TRANSPORT
for n in 2 4; do
  DLI_SHARE_GPU=1 DLI_WATCHDOG_S=120 timeout -k 10 500 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2962$n \
      bench.py --gpus $n --steps 5 --warmup 2 --batch-per-mb 64 --prompt-len 256 > gpurun_out/rehearsal_pp${n}_default.log 2>&1
  rc=$?; grep '^{' gpurun_out/rehearsal_pp${n}_default.log | tail -1 > gpurun_out/rehearsal_pp${n}_default.json
  echo "pp$n rc=$rc $(cut -c1-300 gpurun_out/rehearsal_pp${n}_default.json)"
  [ $rc -eq 0 ] || exit $rc
done
