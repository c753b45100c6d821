#!/bin/bash
# One GPU verification round: tests -> smoke -> bench.  Stops at the first crash/timeout.
# Usage: scripts/gpu_round.sh [bench args...]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m distributed_llm_inference._build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed (rc=$rc); stopping"; exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1200 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
