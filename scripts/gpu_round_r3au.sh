# Round-3 GPU round AU: fp8 GEMV with 8 k-steps of loads in flight (DLI_GEMV_U8=1) vs 4, batch-1 fp8 bench
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
for u in 1 0 1 0; do
  DLI_GEMV_U8=$u timeout -k 10 600 python -u bench.py --fp8 --batch-per-mb 1 --steps 20 --json-out gpurun_out/results/fp8_b1_u$u.json > gpurun_out/results/fp8_b1_u$u.log 2>&1 || { tail -20 gpurun_out/results/fp8_b1_u$u.log; exit 1; }
  echo "fp8 b1 U8=$u $(python -c "import json;d=json.load(open('gpurun_out/results/fp8_b1_u$u.json'));print(d['value'], d['ms_per_step'])")"
done
