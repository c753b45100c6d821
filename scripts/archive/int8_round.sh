#!/bin/bash
# LLM.int8 bench line + rocprofv3 kernel breakdown (one MI355X).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --int8 > gpurun_out/bench_int8.log 2>&1 || { tail -20 gpurun_out/bench_int8.log; exit 1; }
tail -1 gpurun_out/bench_int8.log
bash scripts/archive/prof_int8.sh
