# Round-3 GPU round AH: group size of the grouped tile order at 8192^3 (DLI_GEMM_GM)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_env_ab.py --env DLI_GEMM_GM --vals 8,4,16,2 --rounds 7 \
    --shapes square8k --out gpurun_out/gemm_gm_ab.json > gpurun_out/ah_gm.log 2>&1 || { tail -30 gpurun_out/ah_gm.log; exit 1; }
cat gpurun_out/ah_gm.log
