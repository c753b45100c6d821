# fp8 (config 5 per GPU) routing A/B of gemm4 vs gemm_tile per projection (KernelPolicy.fp8_gemm4),
# same box, interleaved; optional fp8 KV.  Usage: bash scripts/fp8_gemm4_ab.sh [extra bench args]
set -u
mkdir -p gpurun_out/fp8ab
export TMPDIR=/tmp
for pol in none gate_up gate_up+down all none; do
  timeout -k 10 400 python bench.py --fp8 --steps 20 --warmup 5 --kernels fp8_gemm4=$pol "$@" \
      > gpurun_out/fp8ab/$pol.log 2>&1 || { echo "bench $pol failed"; tail -20 gpurun_out/fp8ab/$pol.log; exit 1; }
  grep '^{' gpurun_out/fp8ab/$pol.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pol', d['value'], d['ms_per_step'])"
done
