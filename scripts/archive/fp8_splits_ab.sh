#!/bin/bash
# fp8 + fp8 KV bench: split-K cap (DLI_TILE_MAX_SPLITS) 8 (default heuristic) vs 3 vs 2, alternating
set -o pipefail
mkdir -p gpurun_out/fp8sp
for i in 1 2; do
  for s in 8 3 2; do
    DLI_TILE_MAX_SPLITS=$s timeout -k 10 400 python -u bench.py --fp8 --kv-fp8 --json-out gpurun_out/fp8sp/s${s}_$i.json > gpurun_out/fp8sp/s${s}_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/fp8sp/s${s}_$i.log; exit 1; }
    echo "max_splits=$s run $i: $(python -c "import json;d=json.load(open('gpurun_out/fp8sp/s${s}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
