# Round-3 GPU round AC: MFMA issue order in the bf16 quadrant (DLI_GEMM_ORDER=1: weight fragment
# repeated back to back) - isolated A/B, then in-step A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_env_ab.py --env DLI_GEMM_ORDER --vals 0,1 --rounds 7 \
    --shapes gate_up_swiglu,down_s4,qkv_s3,o_s4 --out gpurun_out/gemm_order_ab.json > gpurun_out/ac_order.log 2>&1 \
    || { tail -30 gpurun_out/ac_order.log; exit 1; }
cat gpurun_out/ac_order.log
timeout -k 10 300 python -u scripts/sample_probe.py > gpurun_out/ac_sample.log 2>&1 || { tail -30 gpurun_out/ac_sample.log; exit 1; }
cat gpurun_out/ac_sample.log
for r in 1 0 0 1; do
  DLI_GEMM_ORDER=$r timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/ac_order$r.json > gpurun_out/ac_order$r.log 2>&1 || { tail -20 gpurun_out/ac_order$r.log; exit 1; }
  echo "bf16 ORDER=$r $(python -c "import json;d=json.load(open('gpurun_out/ac_order$r.json'));print(d['value'], d['ms_per_step'])")"
done
