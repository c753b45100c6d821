set -u
mkdir -p gpurun_out/r6pf
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill" > gpurun_out/r6pf/tests.log 2>&1 || { tail -30 gpurun_out/r6pf/tests.log; exit 1; }
tail -2 gpurun_out/r6pf/tests.log
ARMS="base nostag prio base nostag" QBS="2" bash scripts/prefill_so_ab.sh
