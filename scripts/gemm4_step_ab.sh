#!/bin/bash
# In-step A/B of the decode projections: gemm_tile (DLI_GEMM4=0) vs gemm4 (DLI_GEMM4=1, default),
# bench.py back to back, interleaved twice; extra bench.py arguments (e.g. --fp8) in $1
set -u
mkdir -p gpurun_out/ab
BARGS="${1:-}"
TAG="$(echo "$BARGS" | tr -d ' -')"
for rep in 1 2; do
  for arm in tile gemm4; do
    if [ $arm = gemm4 ]; then export DLI_GEMM4=1; else export DLI_GEMM4=0; fi
    timeout -k 10 400 python3 -u bench.py $BARGS --json-out gpurun_out/ab/${arm}${TAG}_$rep.json > gpurun_out/ab/${arm}${TAG}_$rep.log 2>&1 || { tail -20 gpurun_out/ab/${arm}${TAG}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/${arm}${TAG}_$rep.json'));print('$arm $TAG', $rep, d['value'], d['ms_per_step'])"
  done
done
