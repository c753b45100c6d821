# Round-3 GPU round I: A/B of gate|up on hipBLASLt + separate SwiGLU vs the tile kernel with the
# fused epilogue (default bench, interleaved), and a kernel trace of B=1 decode attention.
set -u
mkdir -p gpurun_out/prof_attn_b1
export TMPDIR=/tmp
timeout -k 10 150 python -u scripts/hwq_probe.py > gpurun_out/hwq_probe.log 2>&1 || { tail -20 gpurun_out/hwq_probe.log; exit 1; }
cat gpurun_out/hwq_probe.log
for r in 1 2; do
  for v in 1 0; do
    DLI_GATEUP_TILE=$v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/bench_gu$v.log 2>&1 || { tail -20 gpurun_out/bench_gu$v.log; exit 1; }
    echo "gate_up_tile=$v $(grep '^{' gpurun_out/bench_gu$v.log | tail -1)" | tee -a gpurun_out/gateup_ab.txt
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_attn_b1 \
    -o attn -- python3 $GRAFT_REPO_ROOT/scripts/attn_bench.py --cases=1x8192,1x600,1x32768 \
    > $GRAFT_REPO_ROOT/gpurun_out/prof_attn_b1.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_attn_b1.log; exit 1; }
tail -4 $GRAFT_REPO_ROOT/gpurun_out/prof_attn_b1.log
