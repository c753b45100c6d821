# In-step A/B of KernelPolicy overrides on one box, interleaved (list the baseline first and
# last).  Usage: TAG=name POLS="gemm4_decode_sched=6 gemm4_decode_sched=9 gemm4_decode_sched=6" \
#                bash scripts/policy_ab.sh [extra bench args, e.g. --fp8 --kv-fp8]
set -u
TAG=${TAG:-ab}
POLS=${POLS:?POLS: space-separated --kernels specs}
out=gpurun_out/$TAG
mkdir -p $out
export TMPDIR=/tmp
n=0
for pol in $POLS; do
  n=$((n + 1))
  log=$out/$n-$pol.log
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --kernels "$pol" "$@" > "$log" 2>&1 \
      || { echo "bench $pol failed"; tail -20 "$log"; exit 1; }
  grep '^{' "$log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$pol', d['value'], d['ms_per_step'])"
done
