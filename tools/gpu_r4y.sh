#!/bin/bash
# MN-major one-wave-per-SIMD weight-gradient tile (120): numerics, then timing against the table.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4y
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_4m_gpu.py -x -q -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "passed|failed|Error|^E " $OUT/t.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u benchmarks/gemm_tile_probe.py --rounds 5 --tiles=-1,120 \
  --ops conv2_wgrad,conv3_wgrad,conv4_wgrad,conv5_wgrad,vgg.c1_2_wgrad,vgg.c2_2_wgrad,vgg.c3_2_wgrad,vgg.c4_2_wgrad,vgg.c5_wgrad \
  > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cut -c1-300 $OUT/probe.jsonl
timeout -k 10 300 python -u -m pytest tests/test_fused_sgd_gpu.py -x -q -rfE --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/sgd.log 2>&1; echo "sgd tests rc=$?"; tail -1 $OUT/sgd.log
for b in 256 32; do timeout -k 10 300 python bench.py --batch $b --steps 30 --warmup 10 2>/dev/null | cut -c1-160; done
