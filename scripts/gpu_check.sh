#!/bin/bash
# One verification call on the MI355X: the GPU test files given as arguments (default: all of
# tests/ marked gpu), then the batch-1 whole-step profiles (scripts/prof_b1.sh).  Every GPU step
# has its own time limit and the steps are chained, so a failure ends the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
files="${*:-tests}"
timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
