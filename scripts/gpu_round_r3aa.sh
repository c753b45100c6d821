# Round-3 GPU round AA: the whole GPU suite + smoke on the current tree
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/aa_gpu_all.log 2>&1
rc=$?; tail -5 gpurun_out/aa_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/aa_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/aa_smoke.log; exit $rc
