# One-half-tile-per-phase DMA schedule (DLI_TILE_EVEN_DMA=1) vs the default: correctness (GEMM
# tests run 3x with the variant), isolated timing, then bench.py A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  DLI_TILE_EVEN_DMA=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread -k "tile" > gpurun_out/even_tests_$i.log 2>&1 || { tail -20 gpurun_out/even_tests_$i.log; exit 1; }
  tail -1 gpurun_out/even_tests_$i.log
done
for e in 0 1; do
  DLI_TILE_EVEN_DMA=$e timeout -k 10 300 python -u scripts/prefill_gateup_probe.py > gpurun_out/even_probe_$e.log 2>&1 || exit 1
  echo "even=$e"; tail -2 gpurun_out/even_probe_$e.log
done
for e in 1 0 1 0; do
  DLI_TILE_EVEN_DMA=$e timeout -k 10 600 python -u bench.py --json-out gpurun_out/even_$e.json > gpurun_out/even_$e.log 2>&1 || exit 1
  echo "bench even=$e $(python -c "import json;d=json.load(open('gpurun_out/even_$e.json'));print(d['value'], d['ms_per_step'])")"
done
