# Round-3 GPU round M: the whole GPU test suite, then the default 1-GPU bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -q --maxfail=15 --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/t_m_all.log 2>&1 || { tail -30 gpurun_out/t_m_all.log; exit 1; }
tail -3 gpurun_out/t_m_all.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_m.log 2>&1 || { tail -20 gpurun_out/bench_m.log; exit 1; }
grep '^{' gpurun_out/bench_m.log | tail -1
