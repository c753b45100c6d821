# Round-3 GPU round V (re-entry): sanity bench of the restored tree; hipBLASLt kernel identity
# (macro tile / MFMA / VGPR / LDS) on the gate|up and square shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/v_bench.json 2> gpurun_out/v_bench.err \
    || { tail -30 gpurun_out/v_bench.err; exit 1; }
cat gpurun_out/v_bench.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/v_blaslt -o blaslt -- \
    python3 $GRAFT_REPO_ROOT/scripts/blaslt_gateup_probe.py > $GRAFT_REPO_ROOT/gpurun_out/v_blaslt.log 2>&1 \
    || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/v_blaslt.log; exit 1; }
tail -3 $GRAFT_REPO_ROOT/gpurun_out/v_blaslt.log
