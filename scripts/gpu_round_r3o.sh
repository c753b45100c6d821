# Round-3 GPU round O: gate|up on the tile kernel with the fused SwiGLU epilogue (default) vs the
# plain bf16 store + separate SwiGLU pass, interleaved on one box.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in 1 plain; do
    DLI_GATEUP_TILE=$v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/bench_gup_$v.log 2>&1 || { tail -20 gpurun_out/bench_gup_$v.log; exit 1; }
    echo "gate_up_tile=$v $(grep '^{' gpurun_out/bench_gup_$v.log | tail -1 | cut -c1-200)" | tee -a gpurun_out/gateup_plain_ab.txt
  done
done
