# one PMC pass over the prefill32 microbench (4 x 4096 causal, qb 2)
set -u
mkdir -p gpurun_out/r6p32
export TMPDIR=/tmp
cd /tmp && CASES=4x4096x0 QB=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmcpf -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6p32/pmc.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py /tmp/pmcpf > gpurun_out/r6p32/pmc_prefill.txt 2>&1
cat gpurun_out/r6p32/pmc_prefill.txt
