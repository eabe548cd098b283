#!/bin/bash
# VGG-16 b64 conv weight-gradient: register kernel vs forced LDS-DMA tiles, standalone.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/gemm_glds_bench.py --iters 10 \
  --ops ${OPS:-vgg.c1_2_wgrad,vgg.c2_1_wgrad,vgg.c2_2_wgrad,vgg.c3_1_wgrad,vgg.c3_2_wgrad,vgg.c4_1_wgrad,vgg.c4_2_wgrad,vgg.c5_wgrad} \
  --tiles ${TILES:-1,7,10,13,17,21,30,34,40,50} > gpurun_out/vgg_wgrad.jsonl 2> gpurun_out/vgg_wgrad.err
rc=$?; cat gpurun_out/vgg_wgrad.jsonl; exit $rc
