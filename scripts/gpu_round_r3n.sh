# Round-3 GPU round N: refreshed decode-step kernel breakdowns (bf16, fp8) and PMC passes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/prof_default.sh || exit $?
bash scripts/pmc_decode.sh || exit $?
mkdir -p gpurun_out/prof_floor
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_floor -o floor \
    -- python3 $GRAFT_REPO_ROOT/scripts/launch_floor_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_floor.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_floor.log; exit 1; }
