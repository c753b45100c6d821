# bf16 headline (N=1, 512 x 512) knob re-check on the final round-6 tree, one box, default first
# and last: stream-K tail, gemm4 decode schedule 6 vs the default 8.
set -u
out=gpurun_out/r6bf16knobs
mkdir -p $out
export TMPDIR=/tmp
n=0
for pol in default stream_k_tail=1 gemm4_decode_sched=6 default; do
  n=$((n + 1))
  log=$out/$n-$pol.log
  k=""; [ "$pol" = default ] || k="--kernels $pol"
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 $k > $log 2>&1 \
    || { echo "bench $pol failed"; tail -20 $log; exit 1; }
  grep '^{' $log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pol', d['value'], d['ms_per_step'])"
done
