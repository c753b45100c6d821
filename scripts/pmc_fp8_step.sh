# PMC of the kernels the DEFAULT fp8 decode step runs: two passes (SQ + GRBM;
# TCC fetch) over bench.py --fp8 [--kv-fp8] with a short decode (64-token prompts, one prefill
# chunk: the decode GEMMs have the headline shapes, M = 512 rows), summarised per dli:: kernel
set -u
out=gpurun_out/r6pmc
mkdir -p $out
export TMPDIR=/tmp
for kv in "--kv-fp8" ""; do
  tag=fp8${kv:+_fp8kv}
  rm -rf $GRAFT_REPO_ROOT/$out/raw_${tag}_1 $GRAFT_REPO_ROOT/$out/raw_${tag}_2
  cd /tmp && timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$out/raw_${tag}_1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --fp8 $kv --steps 3 --warmup 1 --prompt-len 64 --max-batched-tokens 32768 > $GRAFT_REPO_ROOT/$out/${tag}_pass1.log 2>&1 || exit $?
  cd /tmp && timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$out/raw_${tag}_2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --fp8 $kv --steps 3 --warmup 1 --prompt-len 64 --max-batched-tokens 32768 > $GRAFT_REPO_ROOT/$out/${tag}_pass2.log 2>&1 || exit $?
  cd $GRAFT_REPO_ROOT && python3 scripts/pmc_summary.py $GRAFT_REPO_ROOT/$out/raw_${tag}_1 $GRAFT_REPO_ROOT/$out/raw_${tag}_2 > $out/pmc_${tag}_decode_kernels.txt 2>&1 || exit $?
  rm -rf $GRAFT_REPO_ROOT/$out/raw_${tag}_1 $GRAFT_REPO_ROOT/$out/raw_${tag}_2   # (gpurun copies <= 64 MiB back)
  grep -A14 "gemm4_kernel\|gemm_tile_kernel" $out/pmc_${tag}_decode_kernels.txt | head -80
done
