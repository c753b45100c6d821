set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread -k "stream_k or tile" > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/sk_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/gemm_sk_bench.py > gpurun_out/sk_bench.log 2>&1
rc=$?; echo "skbench rc=$rc"; cat gpurun_out/sk_bench.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_sk.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench_sk.log
exit $rc
