#!/bin/bash
# Eager PyTorch-ROCm GoogLeNet / VGG-16 throughput for the comparison table.
set -o pipefail
OUT=gpurun_out/${1:-tm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/torch_models.py --model inception_v1 --batch 128 > $OUT/torch_inception.json 2> $OUT/torch_inception.err || { echo "torch inception failed"; tail -20 $OUT/torch_inception.err; exit 1; }
cat $OUT/torch_inception.json
timeout -k 10 300 python -u benchmarks/torch_models.py --model vgg16 --batch 64 > $OUT/torch_vgg16.json 2> $OUT/torch_vgg16.err || { echo "torch vgg failed"; tail -20 $OUT/torch_vgg16.err; exit 1; }
cat $OUT/torch_vgg16.json
timeout -k 10 300 python -u bench.py --model vgg16 --batch 64 --steps 20 --warmup 5 > $OUT/bench_vgg16.json 2> $OUT/bench_vgg16.err || { echo "vgg bench failed"; tail -20 $OUT/bench_vgg16.err; exit 1; }
cat $OUT/bench_vgg16.json
