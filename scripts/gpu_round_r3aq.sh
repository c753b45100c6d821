# Round-3 GPU round AQ: whole GPU suite + smoke after the fp8 GEMV dispatch
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/aq_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/aq_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/aq_smoke.log 2>&1 || { tail -5 gpurun_out/aq_smoke.log; exit 1; }
tail -1 gpurun_out/aq_smoke.log
