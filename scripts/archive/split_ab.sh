set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for ms in 8 2 1 8 2; do
  DLI_TILE_MAX_SPLITS=$ms timeout -k 10 600 python -u bench.py --json-out gpurun_out/split$ms.json > gpurun_out/split$ms.log 2>&1 || exit $?
  echo "max_splits=$ms $(python -c "import json;d=json.load(open('gpurun_out/split$ms.json'));print(d['value'], d['ms_per_step'])")"
done
