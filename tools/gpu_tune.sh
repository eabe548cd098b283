#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune
timeout -k 10 1000 python -u benchmarks/tune_db.py --models alexnet:256,alexnet:128,alexnet:64,alexnet:32,inception_v1:128,inception_v1:64,vgg16:64,vgg16:32,mnist_conv:100,bowl:64 --out gpurun_out/tune/glds_tune_gfx950.json > gpurun_out/tune/tune.log 2>&1 || { tail -20 gpurun_out/tune/tune.log; exit 1; }
tail -3 gpurun_out/tune/tune.log
