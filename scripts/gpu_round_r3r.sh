# Round-3 GPU round R: 16-byte RoPE kernel - identity tests, then bench A/B (interleaved).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k rope \
    > gpurun_out/t_r_rope.log 2>&1 || { tail -30 gpurun_out/t_r_rope.log; exit 1; }
tail -2 gpurun_out/t_r_rope.log
for r in 1 2; do
  for v in 1 0; do
    DLI_ROPE_V8=$v timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/bench_rope$v.log 2>&1 || { tail -20 gpurun_out/bench_rope$v.log; exit 1; }
    echo "rope_v8=$v $(grep '^{' gpurun_out/bench_rope$v.log | tail -1 | cut -c1-200)" | tee -a gpurun_out/rope_v8_ab.txt
  done
done
