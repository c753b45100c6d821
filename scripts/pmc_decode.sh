# Two PMC passes (SQ + GRBM; TCC fetch) over scripts/pmc_decode_kernels.py, summarised per kernel
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/pmc1 /tmp/pmc2
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmc1 -o run -- python3 scripts/pmc_decode_kernels.py > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d /tmp/pmc2 -o run -- python3 scripts/pmc_decode_kernels.py > gpurun_out/pmc2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py /tmp/pmc1 /tmp/pmc2 > gpurun_out/pmc_decode_kernels.txt 2>&1 || exit $?
cat gpurun_out/pmc_decode_kernels.txt
