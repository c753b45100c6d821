#!/bin/bash
# fp8 / int8 GEMV: norm-prologue loads issued before the pre-issued weight group, unconditional
# (clamped) weight / x loads.  GEMV numerics tests, then old (ab_old/, the base commit built
# separately) vs new interleaved on one box: GEMV stream rates and batch-1 benches.
set -u
mkdir -p gpurun_out/rpre
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_layer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "skinny or gemv or 8bit or norm or decode_layer or rope" > gpurun_out/rpre/tests.log 2>&1 || { tail -30 gpurun_out/rpre/tests.log; exit 1; }
tail -1 gpurun_out/rpre/tests.log
(cd ab_old && timeout -k 10 300 python3 -u scripts/gemv_bw.py fp8 > $GRAFT_REPO_ROOT/gpurun_out/rpre/bw_old.txt 2>&1) || { tail -5 gpurun_out/rpre/bw_old.txt; exit 1; }
timeout -k 10 300 python3 -u scripts/gemv_bw.py fp8 > gpurun_out/rpre/bw_new.txt 2>&1 || { tail -5 gpurun_out/rpre/bw_new.txt; exit 1; }
grep fp8 gpurun_out/rpre/bw_old.txt gpurun_out/rpre/bw_new.txt
run() {  # tag dir flag
  local tag=$1 dir=$2 flag=$3
  (cd $dir && timeout -k 10 300 python3 -u bench.py $flag --batch-per-mb 1 --steps 20 --warmup 3 --json-out $GRAFT_REPO_ROOT/gpurun_out/rpre/$tag.json > $GRAFT_REPO_ROOT/gpurun_out/rpre/$tag.log 2>&1) || { tail -20 gpurun_out/rpre/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/rpre/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run fp8_old1 ab_old --fp8 && run fp8_new1 . --fp8 && run fp8_old2 ab_old --fp8 && run fp8_new2 . --fp8 && run int8_old ab_old --int8 && run int8_new . --int8 
