# Round-3 GPU round D: non-temporal K/V decode A/B (microbench + default bench), clean IPC PP=8
# rehearsal (every sequence fits), default-bench rocprofv3 breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for nt in 0 1 0 1; do
  DLI_KV_NT=$nt timeout -k 10 200 python -u scripts/attn_bench.py --cases=512x600,256x2048,64x4096 \
      > gpurun_out/attn_nt$nt.log 2>&1 || exit $?
  echo "nt=$nt $(grep "'B'" gpurun_out/attn_nt$nt.log | tr '\n' ' ')" | tee -a gpurun_out/nt_ab.txt
done
for nt in 0 1 0 1; do
  DLI_KV_NT=$nt timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
      > gpurun_out/bench_nt$nt.log 2>&1 || exit $?
  echo "nt=$nt $(grep '^{' gpurun_out/bench_nt$nt.log | tail -1 | cut -c1-200)" | tee -a gpurun_out/nt_ab.txt
done
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread \
    tests/test_multiproc_gpu.py -k "deadline" > gpurun_out/t_r3d.log 2>&1
rc=$?; tail -2 gpurun_out/t_r3d.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/rehearsal_pp8_ipc.sh || exit $?
exit 0
