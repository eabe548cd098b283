#!/bin/bash
# few-channel first-layer kernel: numerics, then model A/B (GoogLeNet, VGG-16), IO throughput.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fewc or conv_forward" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b/fewc.log 2>&1
rc=$?; tail -12 gpurun_out/r3b/fewc.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/diag_conv1c3.py > gpurun_out/r3b/diag_c3.log 2>&1; rc=$?; cat gpurun_out/r3b/diag_c3.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh inception_v1 128 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3b/ab_fewc_inc.jsonl || exit 1
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3b/ab_fewc_vgg.jsonl || exit 1
D=/tmp/cxxnet_io_data
timeout -k 10 400 python -u benchmarks/io_throughput.py --dir $D --n 4096 --workers 8,16 --batches 16 \
    --iters imgbin --modes native,process > gpurun_out/r3b/io_decode.jsonl 2> gpurun_out/r3b/io_decode.err || { tail gpurun_out/r3b/io_decode.err; exit 1; }
cat gpurun_out/r3b/io_decode.jsonl
timeout -k 10 400 python -u benchmarks/io_throughput.py --dir $D --workers 16 --batches 24 \
    --iters imgbin --modes native --train alexnet > gpurun_out/r3b/io_train.jsonl 2> gpurun_out/r3b/io_train.err || { tail gpurun_out/r3b/io_train.err; exit 1; }
cat gpurun_out/r3b/io_train.jsonl
