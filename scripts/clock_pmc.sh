# Effective shader clock per kernel (GRBM_GUI_ACTIVE cycles / kernel duration) in the decode step,
# with and without the stream-K tail.  One counter pass per run (no trace domains besides kernels).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sk in 0 1; do
  rm -rf /tmp/pmc_sk$sk
  DLI_TILE_SK=$sk timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/pmc_sk$sk -o run -- python3 bench.py --steps 3 --warmup 1 --no-graphs > gpurun_out/pmc_sk$sk.log 2>&1 || exit $?
  find /tmp/pmc_sk$sk -name "*.csv" > gpurun_out/pmc_sk${sk}_files.txt
  python3 scripts/clock_summary.py /tmp/pmc_sk$sk > gpurun_out/pmc_sk${sk}_clock.txt 2>&1 || exit $?
  cat gpurun_out/pmc_sk${sk}_clock.txt
done
