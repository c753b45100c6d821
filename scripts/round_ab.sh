# Same-box A/B of this tree against an older tree extracted and built under tools_bin/<name>
# (git archive <commit> | tar -x -C tools_bin/<name>; build it there): interleaved bench runs.
# Usage: OLD=r4tree CFGS="bf16 fp8 fp8kv" bash scripts/round_ab.sh
set -u
OLD=${OLD:?OLD: tree under tools_bin}
CFGS=${CFGS:-"bf16 fp8kv fp8"}
out=gpurun_out/round_ab
mkdir -p $out
export TMPDIR=/tmp
args() { case $1 in bf16) echo "";; fp8) echo "--fp8";; fp8kv) echo "--fp8 --kv-fp8";; esac; }
for cfg in $CFGS; do
  for arm in new old new old; do
    n=$(ls $out | wc -l)
    log=$PWD/$out/$n-$cfg-$arm.log
    if [ $arm = new ]; then dir=.; else dir=tools_bin/$OLD; fi
    (cd $dir && timeout -k 10 400 python bench.py --steps 20 --warmup 5 $(args $cfg) > "$log" 2>&1) \
        || { echo "$cfg $arm failed"; tail -20 "$log"; exit 1; }
    grep '^{' "$log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg $arm', d['value'], d['ms_per_step'])"
  done
done
