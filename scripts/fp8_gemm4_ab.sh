# fp8 (config 5 per GPU) routing A/B of gemm4 vs gemm_tile per projection (KernelPolicy.fp8_gemm4),
# same box, interleaved (the baseline first and last); optional fp8 KV.
# Usage: [TAG=_kv8] [POLS="none all none"] bash scripts/fp8_gemm4_ab.sh [extra bench args]
set -u
TAG=${TAG:-}
POLS=${POLS:-"none gate_up gate_up+down all none"}
out=gpurun_out/fp8ab$TAG
mkdir -p $out
export TMPDIR=/tmp
n=0
for pol in $POLS; do
  n=$((n + 1))
  log=$out/$n-$pol.log
  timeout -k 10 400 python bench.py --fp8 --steps 20 --warmup 5 --kernels fp8_gemm4=$pol "$@" \
      > $log 2>&1 || { echo "bench $pol failed"; tail -20 $log; exit 1; }
  grep '^{' $log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pol', d['value'], d['ms_per_step'])"
done
