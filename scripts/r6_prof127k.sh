# rocprofv3 kernel statistics of a Llama-3.1-70B bf16 127k-token prompt (TTFT attribution: the
# prefill32 attention vs the hipBLASLt projections) on the final round-6 tree.
set -u
out=gpurun_out/r6p127
mkdir -p $out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 130048 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 scripts/stats_top.py $(find $out/prof -name "*kernel_stats.csv" | head -1) > $out/prof127k_kernel_stats_top.txt && head -12 $out/prof127k_kernel_stats_top.txt
rm -rf $out/prof/*/*kernel_trace.csv
