# Round-3 GPU round AB: sampler timing on the LM-head shape
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sample_probe.py > gpurun_out/ab_sample.log 2>&1 || { tail -30 gpurun_out/ab_sample.log; exit 1; }
cat gpurun_out/ab_sample.log
