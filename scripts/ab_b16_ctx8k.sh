set -u
out=gpurun_out/ab16
mkdir -p $out
for arm in new old new old; do
  n=$(ls $out | wc -l)
  log=$PWD/$out/$n-$arm.log
  if [ $arm = new ]; then dir=.; else dir=tools_bin/r4tree; fi
  (cd $dir && timeout -k 10 400 python bench.py --batch-per-mb 16 --prompt-len 8192 --steps 10 > "$log" 2>&1) || { echo "$arm failed"; tail -20 "$log"; exit 1; }
  grep '^{' "$log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])"
done
