#!/bin/bash
# Final-tree check on one MI355X: every GPU test, smoke(), the default bench (driver's N = 1 call).
set -u
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests_all.log 2>&1 || { tail -30 gpurun_out/final/gpu_tests_all.log; exit 1; }
tail -2 gpurun_out/final/gpu_tests_all.log
timeout -k 10 300 python3 -u __graft_entry__.py smoke > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -20 gpurun_out/final/bench_default.err; exit 1; }
tail -1 gpurun_out/final/bench_default.json
