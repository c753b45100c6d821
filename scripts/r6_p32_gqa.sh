# prefill32 for any GQA group: oracle tests, then the microbench against attention.hip's kernel
# for MHA (Llama-2 shape, 32 / 32) and Qwen2-7B's group of 7 (28 / 4)
set -u
out=gpurun_out/r6gqa
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "prefill or attn" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for hk in "32 32" "28 4" "16 8"; do
  set -- $hk
  for m in 1 0; do
    NH=$1 NKV=$2 CASES=4x4096x0,32x512x0,1x2048x6144 TAG=gqa$1_$2_m$m DLI_KERNELS=prefill_m32=$m timeout -k 10 200 python -u scripts/attn_prefill_bench.py > $out/b_$1_$2_m$m.txt 2>&1 || { tail -5 $out/b_$1_$2_m$m.txt; exit 1; }
    grep TFLOPs $out/b_$1_$2_m$m.txt
  done
done
