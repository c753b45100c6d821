# Round-3 GPU round AI: refreshed PMC passes of the decode kernels on the final tree
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/pmc_decode.sh || exit $?
