# Round-3 GPU round: whole GPU suite, then the 8-rank IPC rehearsal of the default PP=8 path,
# then the default 1-GPU bench.  A crash / abort / timeout ends the script (no further GPU step);
# plain test failures (rc 1) still let the later steps run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/t_gpu_all.log 2>&1
rc=$?; tail -4 gpurun_out/t_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/rehearsal_pp8_ipc.sh
rc2=$?
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1
rc3=$?; tail -1 gpurun_out/bench_n1.log
[ $rc3 -ne 0 ] && exit $rc3
exit $rc
