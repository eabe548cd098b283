#!/bin/bash
# VGG-16: in-step tuning of conv forward / data-gradient signatures over the persistent halo tiles,
# then an interleaved A/B of the shipped table against the tuned one (same box)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4aj
mkdir -p $OUT
timeout -k 10 600 python3 -u benchmarks/step_tune.py --model vgg16 --batch 64 --ops cf,cd --cands 132,133 --out $OUT/vgg_ps.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "key|final" $OUT/tune.log | tail -40
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_ps.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_ps.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_ps.json" > $OUT/ab.jsonl || exit 1
cat $OUT/ab.jsonl
