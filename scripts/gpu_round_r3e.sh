# Round-3 GPU round E: the IPC PP=8 rehearsal (b32 x p256) with per-thread / per-channel records,
# then a PP=4 variant of the same config.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/rehearsal_pp8_ipc.sh
rc=$?
cp gpurun_out/rehearsal_pp8_ipc.log gpurun_out/rehearsal_pp8_ipc_e1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DLI_SHARE_GPU=1 DLI_TRANSPORT=ipc DLI_WATCHDOG_S=120 timeout -k 10 600 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29617 \
    bench.py --gpus 4 --steps 5 --warmup 2 --batch-per-mb 32 --prompt-len 256 > gpurun_out/rehearsal_pp4_ipc.log 2>&1
rc2=$?; grep '^{' gpurun_out/rehearsal_pp4_ipc.log | tail -1 | cut -c1-300; exit $(( rc > rc2 ? rc : rc2 ))
