set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/gemm_sk_bench.py > gpurun_out/sk_bench2.log 2>&1 || exit $?
tail -3 gpurun_out/sk_bench2.log
for sk in 0 1 0 1; do
  DLI_TILE_SK=$sk timeout -k 10 600 python -u bench.py --json-out gpurun_out/ab_sk$sk.json > gpurun_out/ab_sk$sk.log 2>&1 || exit $?
  echo "SK=$sk $(python -c "import json;d=json.load(open('gpurun_out/ab_sk$sk.json'));print(d['value'], d['ms_per_step'])")"
done
