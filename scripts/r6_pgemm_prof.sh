# kernel stats of the headline prefill with the two large-M GEMM routings
set -u
out=gpurun_out/r6pgemm3
mkdir -p $out
export TMPDIR=/tmp
for pol in 0 2048; do
  cd /tmp && rm -rf /tmp/pp_$pol && DLI_KERNELS=tile_gemm_max_m=$pol timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp_$pol -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$out/p_$pol.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT && python3 scripts/stats_top.py $(find /tmp/pp_$pol -name "*kernel_stats.csv" | head -1) > $out/top_$pol.txt && head -14 $out/top_$pol.txt
done
