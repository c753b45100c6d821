# 32k-token prefill (Llama-3.1-70B bf16, batch 1): large-M projections on hipBLASLt (default)
# vs the hand-written tile kernels (library_gemms=0), same box
set -u
out=gpurun_out/r6pgemm
mkdir -p $out
export TMPDIR=/tmp
for lib in 1 0; do
  DLI_KERNELS=library_gemms=$lib timeout -k 10 500 python -u bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 3 --warmup 1 --json-out $out/lib$lib.json > $out/lib$lib.log 2>&1 || { tail -20 $out/lib$lib.log; exit 1; }
  python -c "import json; d=json.load(open('$out/lib$lib.json')); print('library_gemms=$lib', 'prefill_s', d['prefill_s'], 'tok/s', d['value'])"
done
