# prefill32 on a StreamingLLM sink window (70B heads, W = 4096, 4 sinks) against attention.hip
set -u
out=gpurun_out/r6sink
mkdir -p $out
export TMPDIR=/tmp
for m in 1 0; do
  N_SINK=4 WINDOW=4096 CASES=4x4096x0,1x8192x0,1x2048x6144,32x512x0 TAG=sink_m$m DLI_KERNELS=prefill_m32=$m timeout -k 10 200 python -u scripts/attn_prefill_bench.py > $out/b_m$m.txt 2>&1 || { tail -5 $out/b_m$m.txt; exit 1; }
  grep TFLOPs $out/b_m$m.txt
done
