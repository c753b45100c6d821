# two more PMC passes over the prefill32 microbench (4 x 4096 causal, qb 2): issue mix and LDS
set -u
mkdir -p gpurun_out/r6p32
export TMPDIR=/tmp
cd /tmp
CASES=4x4096x0 QB=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmcA -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6p32/pmcA.log 2>&1 || exit $?
CASES=4x4096x0 QB=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmcB -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6p32/pmcB.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py /tmp/pmcA > gpurun_out/r6p32/pmc_prefill_A.txt 2>&1 && python3 scripts/pmc_summary.py /tmp/pmcB > gpurun_out/r6p32/pmc_prefill_B.txt 2>&1
cat gpurun_out/r6p32/pmc_prefill_A.txt gpurun_out/r6p32/pmc_prefill_B.txt
