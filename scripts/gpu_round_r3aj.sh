# Round-3 GPU round AJ: whole GPU suite + smoke on the final tree; B=1 decode attention at short
# contexts (4 merged splits, no combine) and the batch-1 bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/aj_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/aj_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/aj_smoke.log 2>&1 || { tail -5 gpurun_out/aj_smoke.log; exit 1; }
tail -1 gpurun_out/aj_smoke.log
timeout -k 10 300 python -u scripts/attn_bench.py --cases=1x600,1x768,4x600,16x600 > gpurun_out/aj_attn.log 2>&1 || { tail -20 gpurun_out/aj_attn.log; exit 1; }
cat gpurun_out/aj_attn.log
timeout -k 10 300 python -u bench.py --batch-per-mb 1 --steps 20 --json-out gpurun_out/aj_b1.json > gpurun_out/aj_b1.log 2>&1 || { tail -20 gpurun_out/aj_b1.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/aj_b1.json'));print('b1', d['value'], d['ms_per_step'])"
