# rocprofv3 decode breakdowns of KernelPolicy overrides on one box:
# POLS="fp8_gemm4=gate_up fp8_gemm4=all" TAG=name bash scripts/policy_prof.sh [bench args]
set -u
TAG=${TAG:-policy_prof}
POLS=${POLS:?POLS}
out=gpurun_out/$TAG
mkdir -p $out
export TMPDIR=/tmp
n=0
for pol in $POLS; do
  n=$((n + 1))
  rm -rf /tmp/pprof_$n
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pprof_$n -o run -- python3 bench.py --steps 5 --warmup 2 --kernels "$pol" "$@" > $out/$n.log 2>&1 || exit $?
  f=$(find /tmp/pprof_$n -name "*kernel_trace.csv" | head -1)
  python3 scripts/analyze_trace.py "$f" --steps 3 > $out/$n-$pol.breakdown.txt || exit $?
  echo "== $pol"; head -12 $out/$n-$pol.breakdown.txt
done
