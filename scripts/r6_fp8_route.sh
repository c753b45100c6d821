# fp8 + fp8 KV (config 5 per GPU) routing re-check on the final round-6 tree, same box, baseline
# first and last: hipBLASLt for the K = 8192 projections (tile_gemms=0) and gemm4 on down too.
set -u
out=gpurun_out/r6fp8route
mkdir -p $out
export TMPDIR=/tmp
n=0
for pol in default tile_gemms=0 fp8_gemm4=gate_up+down default; do
  n=$((n + 1))
  log=$out/$n-$pol.log
  k=""; [ "$pol" = default ] || k="--kernels $pol"
  timeout -k 10 400 python bench.py --fp8 --kv-fp8 --steps 20 --warmup 5 $k > $log 2>&1 \
    || { echo "bench $pol failed"; tail -20 $log; exit 1; }
  grep '^{' $log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pol', d['value'], d['ms_per_step'])"
done
