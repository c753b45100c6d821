# Round-3 GPU round X: bf16 tile GEMM variants (DLI_GEMM_VAR: NT weight loads, grouped tile order)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/gemm_env_ab.py --env DLI_GEMM_VAR --vals 0,1,2,3 --rounds 7 \
    --out gpurun_out/gemm_var_nt_group_ab.json > gpurun_out/x_var_ab.log 2>&1 \
    || { tail -30 gpurun_out/x_var_ab.log; exit 1; }
cat gpurun_out/x_var_ab.log
