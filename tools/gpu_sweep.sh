#!/bin/bash
# Tile sweep of the LDS-DMA GEMM on AlexNet / VGG-16 ops.  bash tools/gpu_sweep.sh <tag> <ops> <tiles>
set -o pipefail
TAG=$1; OPS=$2; TILES=$3
mkdir -p gpurun_out/sweep
timeout -k 10 900 python benchmarks/gemm_glds_bench.py --iters 20 --ops $OPS --tiles $TILES > gpurun_out/sweep/$TAG.jsonl 2> gpurun_out/sweep/$TAG.err || { echo sweep failed; tail -20 gpurun_out/sweep/$TAG.err; exit 1; }
cat gpurun_out/sweep/$TAG.jsonl
