#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2c
mkdir -p $OUT
timeout -k 10 300 python benchmarks/gemm_ceiling.py --model alexnet > $OUT/ceiling_alexnet.jsonl 2> $OUT/ceiling.err || { echo ceiling failed; tail $OUT/ceiling.err; exit 1; }
timeout -k 10 300 python benchmarks/gemm_ceiling.py --model vgg16 > $OUT/ceiling_vgg16.jsonl 2>> $OUT/ceiling.err || { echo ceiling vgg failed; tail $OUT/ceiling.err; exit 1; }
bash tools/pmc_top.sh top conv2_fwd conv2_dgrad conv2_wgrad conv3_fwd conv3_dgrad conv1_fwd conv1_wgrad fc6_fwd fc6_wgrad fc6_dgrad vgg_c3_2_fwd vgg_c3_2_dgrad vgg_c3_2_wgrad
