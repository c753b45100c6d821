# prefill32 on a Mistral-style sliding window (32 q / 8 kv heads, W = 4096, no sinks) against
# attention.hip's kernel: prompts below and above the window, a chunk on a wrapped ring
set -u
out=gpurun_out/r6win
mkdir -p $out
export TMPDIR=/tmp
for m in 1 0; do
  NH=32 NKV=8 WINDOW=4096 CASES=4x4096x0,1x8192x0,1x2048x6144,32x512x0 TAG=win_m$m DLI_KERNELS=prefill_m32=$m timeout -k 10 200 python -u scripts/attn_prefill_bench.py > $out/b_m$m.txt 2>&1 || { tail -5 $out/b_m$m.txt; exit 1; }
  grep TFLOPs $out/b_m$m.txt
done
