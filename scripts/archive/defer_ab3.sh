set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/defer4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/defer4_tests.log; [ $rc -ne 0 ] && exit $rc
for d in 1 0 1 0; do
  DLI_SPLITK_DEFER=$d timeout -k 10 600 python -u bench.py --json-out gpurun_out/defer4_$d.json > gpurun_out/defer4_$d.log 2>&1 || exit $?
  echo "bf16 defer=$d $(python -c "import json;d=json.load(open('gpurun_out/defer4_$d.json'));print(d['value'], d['ms_per_step'])")"
done
rm -rf /tmp/prof_t
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_t -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_t.log 2>&1 || exit $?
f=$(find /tmp/prof_t -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_t_breakdown.txt || exit $?
head -9 gpurun_out/prof_t_breakdown.txt
