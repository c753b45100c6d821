# Round-3 GPU round AM: final-tree sanity - smoke + default bench (the driver's contract)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/am_smoke.log 2>&1 || { tail -5 gpurun_out/am_smoke.log; exit 1; }
tail -1 gpurun_out/am_smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/am_bench.json 2> gpurun_out/am_bench.err || { tail -20 gpurun_out/am_bench.err; exit 1; }
cat gpurun_out/am_bench.json
