# large-M projections on the tile kernels (new default) vs hipBLASLt above M = 2048 (round-5 rule,
# tile_gemm_max_m=2048), same box: TTFT of 32k-token prompts and the headline bench
set -u
out=gpurun_out/r6pgemm
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $out/gemm_tests.log 2>&1 || { tail -30 $out/gemm_tests.log; exit 1; }
tail -1 $out/gemm_tests.log
run() {  # name, policy, args...
  local name=$1 pol=$2; shift 2
  DLI_KERNELS=$pol timeout -k 10 600 python -u bench.py "$@" --json-out $out/$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  python -c "import json; d=json.load(open('$out/$name.json')); print('$name', 'prefill_s', d['prefill_s'], 'tok/s', d['value'])"
}
for pol in tile_gemm_max_m=0 tile_gemm_max_m=2048; do
  run 70b_32k_$pol $pol --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 3 --warmup 1
  run 70b_fp8_32k_$pol $pol --model llama-3.1-70b --fp8 --batch-per-mb 1 --prompt-len 32768 --steps 3 --warmup 1
  run 8b_32k_$pol $pol --model llama-3-8b --batch-per-mb 1 --prompt-len 32768 --steps 3 --warmup 1
  run headline_$pol $pol --steps 10 --warmup 3
done
