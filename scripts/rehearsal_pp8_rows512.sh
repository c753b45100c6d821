# 8-rank PP=8 host-path rehearsal at the REAL micro-batch size on ONE shared GPU (VERDICT r4 next
# #1a): Llama-3-70B width with 16 layers (2 per stage, so 8 ranks x 9 micro-batches x 512 rows and
# their KV fit one GPU), IPC device transport with the production stream schedule, rotating head,
# graphs pre-captured, watchdog armed.  Device throughput is meaningless (8 ranks share one GPU);
# what is measured is each rank's HOST time per micro-batch step, by phase (runtime/hostclock.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
DLI_SHARE_GPU=1 DLI_TRANSPORT=ipc DLI_WATCHDOG_S=${DLI_WATCHDOG_S:-180} timeout -k 10 1000 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 \
    bench.py --gpus 8 --steps ${STEPS:-10} --warmup 3 --num-layers 16 --batch-per-mb 512 --prompt-len 512 \
    --kv-fp8 --max-batched-tokens 4096 > gpurun_out/rehearsal_pp8_rows512.log 2>&1
rc=$?; grep '^{' gpurun_out/rehearsal_pp8_rows512.log | tail -1 > gpurun_out/rehearsal_pp8_rows512.json
tail -3 gpurun_out/rehearsal_pp8_rows512.log | cut -c1-400; exit $rc
