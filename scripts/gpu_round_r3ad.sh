# Round-3 GPU round AD: decode attention rate vs batch (round structure: 2 workgroups per CU)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/attn_bench.py --cases=128x600,256x600,512x600,1024x600,256x1200,512x1200,2048x600 \
    > gpurun_out/ad_attn.log 2>&1 || { tail -30 gpurun_out/ad_attn.log; exit 1; }
cat gpurun_out/ad_attn.log
