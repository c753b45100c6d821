# prefill32 rework: oracle tests on the in-tree build, then the same-box microbench A/B
# (ARMS: tools_bin/variants/<arm> builds; base = in-tree)
set -u
mkdir -p gpurun_out/r6p32
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefill or attn" > gpurun_out/r6p32/tests.log 2>&1 || { tail -40 gpurun_out/r6p32/tests.log; exit 1; }
tail -3 gpurun_out/r6p32/tests.log
ARMS=${ARMS:-"base"} QBS=${QBS:-"1 2"} TAG=${TAG:-r6p32} bash scripts/prefill_so_ab.sh
