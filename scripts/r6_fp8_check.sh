# fp8 + fp8 KV 127k TTFT regression hunt: warm-up on/off, prefill32 fp8 on/off, fp8 attention bench
set -u
out=gpurun_out/r6f8chk
mkdir -p $out
export TMPDIR=/tmp
KV_FP8=1 CASES=4x4096x0,1x2048x6144 TAG=f8chk timeout -k 10 200 python -u scripts/attn_prefill_bench.py 2>&1 | grep TFLOPs
for pol in warm_library_gemms=0 prefill_m32=0; do
  DLI_KERNELS=$pol timeout -k 10 600 python -u bench.py --model llama-3.1-70b --fp8 --kv-fp8 --batch-per-mb 1 --prompt-len 130048 --steps 2 --warmup 1 --json-out $out/$pol.json > $out/$pol.log 2>&1 || { tail -20 $out/$pol.log; exit 1; }
  python -c "import json; d=json.load(open('$out/$pol.json')); print('$pol prefill_s', d['prefill_s'])"
done
