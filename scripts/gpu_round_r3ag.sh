# Round-3 GPU round AG: per-kernel decode-step breakdowns (bf16, fp8) and the README results sweep
# on the current tree, one box
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/prof_default.sh || exit $?
bash scripts/results_sweep.sh || exit $?
