# the headline prefill (512 x 512-token prompts, 16384-token chunks) and the 32k-token prompt,
# alternating the two GEMM routings twice, same box
set -u
out=gpurun_out/r6pgemm2
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
  for pol in 0 2048; do
    DLI_KERNELS=tile_gemm_max_m=$pol timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --json-out $out/h_${pol}_$i.json > $out/h_${pol}_$i.log 2>&1 || { tail -20 $out/h_${pol}_$i.log; exit 1; }
    DLI_KERNELS=tile_gemm_max_m=$pol timeout -k 10 600 python -u bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 2 --warmup 1 --json-out $out/l_${pol}_$i.json > $out/l_${pol}_$i.log 2>&1 || { tail -20 $out/l_${pol}_$i.log; exit 1; }
    python -c "import json; a=json.load(open('$out/h_${pol}_$i.json')); b=json.load(open('$out/l_${pol}_$i.json')); print('max_m=$pol run $i headline prefill_s', a['prefill_s'], '32k prefill_s', b['prefill_s'])"
  done
done
