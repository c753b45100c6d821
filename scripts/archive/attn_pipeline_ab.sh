#!/bin/bash
# Interleaved same-box A/B of the decode-attention load pipeline fix: ab_old/ = the tree before it
# (built separately), . = with it.  Default bench x2 each, fp8 + fp8 KV x1 each.
set -u
mkdir -p gpurun_out/attnab
export TMPDIR=/tmp
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 400 python3 -u bench.py "$@" --json-out $GRAFT_REPO_ROOT/gpurun_out/attnab/$tag.json > $GRAFT_REPO_ROOT/gpurun_out/attnab/$tag.log 2>&1) || { tail -20 gpurun_out/attnab/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/attnab/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run old1 ab_old && run new1 . && run old2 ab_old && run new2 . && run old_fp8kv ab_old --fp8 --kv-fp8 && run new_fp8kv . --fp8 --kv-fp8
