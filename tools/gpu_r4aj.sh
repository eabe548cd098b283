#!/bin/bash
# Bias loaded once per epilogue: halo numerics, probe of the halo tiles, in-step tuning of VGG-16's
# conv forward / data-gradient signatures over 130-133, A/B of the shipped vs the tuned table, and
# A/B of the pre-epilogue-change tree (_ab/base) vs this tree on AlexNet and GoogLeNet
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4aj
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_gemm_4w_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u benchmarks/gemm_tile_probe.py --ops vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_1_fwd,vgg.c2_2_fwd,vgg.c3_2_fwd --tiles=-1,130,131,132,133 --rounds 5 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cut -c1-330 $OUT/probe.jsonl
timeout -k 10 600 python3 -u benchmarks/step_tune.py --model vgg16 --batch 64 --ops cf,cd --cands 130,131,132,133 --out $OUT/vgg_tuned.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "key|final" $OUT/tune.log | cut -c1-160 | tail -40
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_tuned.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_tuned.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/vgg_tuned.json" > $OUT/ab_table.jsonl || exit 1
cat $OUT/ab_table.jsonl
MODELS="alexnet:256 inception_v1:128" bash tools/gpu_ab_commits.sh _ab/base . _ab/base . || exit 1
cp gpurun_out/ab/ab.jsonl $OUT/ab_tree.jsonl
