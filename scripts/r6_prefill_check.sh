# new prefill kernel: oracle tests, the microbench at qb 1 / 2 with and without it, one PMC pass
set -u
mkdir -p gpurun_out/r6pf
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill" > gpurun_out/r6pf/tests.log 2>&1 || { tail -40 gpurun_out/r6pf/tests.log; exit 1; }
tail -3 gpurun_out/r6pf/tests.log
for qb in 1 2; do
  QB=$qb timeout -k 10 200 python -u scripts/attn_prefill_bench.py > gpurun_out/r6pf/bench_m32_qb$qb.txt 2>&1 || exit $?
  grep TFLOPs gpurun_out/r6pf/bench_m32_qb$qb.txt
done
QB=1 DLI_KERNELS=prefill_m32=0 timeout -k 10 200 python -u scripts/attn_prefill_bench.py > gpurun_out/r6pf/bench_legacy.txt 2>&1 || exit $?
grep TFLOPs gpurun_out/r6pf/bench_legacy.txt
cd /tmp && CASES=4x4096x0 QB=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmcpf -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6pf/pmc.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py /tmp/pmcpf > gpurun_out/r6pf/pmc_prefill.txt 2>&1
cat gpurun_out/r6pf/pmc_prefill.txt
