#!/bin/bash
# gemm4 (one wave per SIMD) vs gemm_tile: bit-exact checks + interleaved timing on the decode shapes
set -u
mkdir -p gpurun_out
timeout -k 10 240 ./tools_bin/gemm4_bench ${1:-7} ${2:-0} > gpurun_out/gemm4_ab.txt 2>&1
rc=$?
cat gpurun_out/gemm4_ab.txt
exit $rc
