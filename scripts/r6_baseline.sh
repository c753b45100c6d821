set -u
mkdir -p gpurun_out/r6base
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6base/bench.json 2> gpurun_out/r6base/bench.err || exit $?
timeout -k 10 200 python -u scripts/attn_prefill_bench.py > gpurun_out/r6base/prefill.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6base/prof_prefill -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6base/prof_prefill.log 2>&1
