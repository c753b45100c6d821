# hop integrity on the GPU: the digest kernel against its reference, then the 8-rank PP=8
# rehearsal on one GPU (IPC device transport, rotating head) with the check on (bench default)
# and off, for the timed ms/step comparison
set -u
out=gpurun_out/r6hop
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "digest" > $out/digest_tests.log 2>&1 || { tail -30 $out/digest_tests.log; exit 1; }
tail -1 $out/digest_tests.log
for hc in 1 0; do
  DLI_HOP_CHECK=$hc bash scripts/rehearsal_pp8_rows512.sh || { echo "rehearsal (hop check $hc) failed"; exit 1; }
  cp gpurun_out/rehearsal_pp8_rows512.log $out/rehearsal_hop$hc.log
  cp gpurun_out/rehearsal_pp8_rows512.json $out/rehearsal_hop$hc.json
  python -c "import json; d=json.load(open('$out/rehearsal_hop$hc.json')); print('hop_check=$hc', d['ms_per_step'], d.get('hop_integrity'), d['transport'])"
done
