# Round-3 GPU round W: k-split bf16 GEMM main loop (DLI_GEMM_KS) - identity + A/B on the decode shapes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_ks_ab.py --rounds 7 > gpurun_out/w_ks_ab.log 2>&1 \
    || { tail -30 gpurun_out/w_ks_ab.log; exit 1; }
cat gpurun_out/w_ks_ab.log
