#!/bin/bash
# New address-free one-wave-per-SIMD GEMM tiles (110-113): numerics, then interleaved timing vs
# tile 21 and hipBLASLt on square and VGG / AlexNet conv shapes.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|Error|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u benchmarks/gemm_tile_probe.py --ops sq8192_fwd,sq4096_fwd,vgg.c4_2_fwd,vgg.c3_2_fwd,vgg.c4_2_dgrad,vgg.c5_fwd,conv3_fwd,conv4_fwd,fc6_fwd --tiles 21,110,111,112,113 --rounds 5 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cut -c1-400 $OUT/probe.jsonl
