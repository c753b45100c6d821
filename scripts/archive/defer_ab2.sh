set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/defer2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/defer2_tests.log; [ $rc -ne 0 ] && exit $rc
for d in 1 0 1 0; do
  DLI_SPLITK_DEFER=$d timeout -k 10 600 python -u bench.py --json-out gpurun_out/defer2_$d.json > gpurun_out/defer2_$d.log 2>&1 || exit $?
  echo "defer=$d $(python -c "import json;d=json.load(open('gpurun_out/defer2_$d.json'));print(d['value'], d['ms_per_step'])")"
done
