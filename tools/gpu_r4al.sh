#!/bin/bash
# VGG-16: in-step tuning of the weight-gradient tiles over the halo widths (140 auto / 141 16 /
# 142 32) and the register split-K kernel, then an interleaved A/B of the shipped vs the tuned table
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4al
mkdir -p $OUT
timeout -k 10 600 python3 -u benchmarks/step_tune.py --model vgg16 --batch 64 --ops cw --cands 99,140,141,142 --out $OUT/vgg_cw.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "key|final" $OUT/tune.log | cut -c1-160 | tail -30
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_cw.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_cw.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_cw.json" > $OUT/ab_table.jsonl || exit 1
cat $OUT/ab_table.jsonl
