#!/bin/bash
# PMC passes (one counter group per run, --kernel-trace only) over the gate|up tile GEMM:
# SwiGLU epilogue vs plain bf16 store, same main loop (scripts/gemm_shape_probe.py cases).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/pmce1 /tmp/pmce2 /tmp/pmce3
P="python3 scripts/gemm_shape_probe.py --only=gate_up_M512_swiglu,gate_up_M512_plain --no-blas"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmce1 -o run -- $P > gpurun_out/pmce1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d /tmp/pmce2 -o run -- $P > gpurun_out/pmce2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d /tmp/pmce3 -o run -- $P > gpurun_out/pmce3.log 2>&1 || exit $?
python3 scripts/pmc_summary.py /tmp/pmce1 /tmp/pmce2 /tmp/pmce3 > gpurun_out/pmc_gemm_epi.txt 2>&1 || exit $?
cat gpurun_out/pmc_gemm_epi.txt
