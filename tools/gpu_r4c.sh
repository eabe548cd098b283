#!/bin/bash
# New GEMM tiles + C++ launch-list executor: numerics, tile timing, foreign-op census, host cost
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gemm_4w_gpu.py tests/test_launch_replay_gpu.py tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|Error|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log
timeout -k 10 400 python -u benchmarks/gemm_tile_probe.py --ops sq8192_fwd,sq4096_fwd,vgg.c4_2_fwd,vgg.c3_2_fwd,vgg.c4_2_dgrad,vgg.c5_fwd,conv3_fwd,conv4_fwd,fc6_fwd --tiles 21,110,111,112,113,114,115 --rounds 5 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cut -c1-300 $OUT/probe.jsonl
timeout -k 10 200 python -u benchmarks/foreign_ops.py --model alexnet --batch 32 > $OUT/foreign.jsonl 2> $OUT/foreign.err || tail -5 $OUT/foreign.err
cut -c1-600 $OUT/foreign.jsonl
for r in 0 1; do CXXNET_LAUNCH_REPLAY=$r timeout -k 10 200 python -u benchmarks/host_overhead.py --batch 32 >> $OUT/host.jsonl 2>> $OUT/host.err || tail -5 $OUT/host.err; done
cat $OUT/host.jsonl
exit $rc
