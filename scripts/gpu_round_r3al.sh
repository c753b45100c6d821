# Round-3 GPU round AL: two whole tiles per workgroup (224 workgroups for gate|up, DLI_GEMM_P2=1)
# vs one (448): isolated shapes, then in-step A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_env_ab.py --env DLI_GEMM_P2 --vals 0,1 --rounds 9 \
    --shapes gate_up_swiglu,plain_M512,gate_up_M300 --out gpurun_out/gemm_p2_ab.json > gpurun_out/al_p2.log 2>&1 \
    || { tail -30 gpurun_out/al_p2.log; exit 1; }
cat gpurun_out/al_p2.log
for r in 1 0 0 1; do
  DLI_GEMM_P2=$r timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --json-out gpurun_out/al_p2_$r.json > gpurun_out/al_p2_$r.log 2>&1 || { tail -20 gpurun_out/al_p2_$r.log; exit 1; }
  echo "bf16 P2=$r $(python -c "import json;d=json.load(open('gpurun_out/al_p2_$r.json'));print(d['value'], d['ms_per_step'])")"
done
