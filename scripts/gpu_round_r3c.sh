# Round-3 GPU round C: new kernel tests, bf16-partials A/B on the default bench, IPC PP=8 rehearsal.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
    -k "custom_mask or bf16_operand_bf16_partials" > gpurun_out/t_r3c.log 2>&1
rc=$?; tail -3 gpurun_out/t_r3c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for parts in 0 1 0 1; do
  DLI_BF16_PARTS=$parts timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
      > gpurun_out/bench_parts$parts.log 2>&1 || exit $?
  echo "parts=$parts $(grep '^{' gpurun_out/bench_parts$parts.log | tail -1 | cut -c1-200)" | tee -a gpurun_out/parts_ab.txt
done
bash scripts/rehearsal_pp8_ipc.sh
exit $?
