# Round-3 GPU round AE: multi-process GPU tests, then the 8-rank default-transport rehearsal
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multiproc_gpu.py \
    > gpurun_out/ae_multiproc.log 2>&1 || { tail -40 gpurun_out/ae_multiproc.log; exit 1; }
tail -2 gpurun_out/ae_multiproc.log
bash scripts/rehearsal_pp8_default.sh
