#!/bin/bash
# IO pipeline throughput on the GPU box (its CPU share), decode alone and feeding AlexNet training.
set -o pipefail
mkdir -p gpurun_out
D=/tmp/cxxnet_io_data
echo "host cpus: $(nproc), affinity: $(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
timeout -k 10 500 python -u benchmarks/io_throughput.py --dir $D --n 4096 --workers 8,16 --batches 16 \
    --iters imgbin --modes process,thread > gpurun_out/io_decode.jsonl 2> gpurun_out/io_decode.err || exit $?
cat gpurun_out/io_decode.jsonl
timeout -k 10 400 python -u benchmarks/io_throughput.py --dir $D --workers 16 --batches 24 \
    --iters imgbin,imgbinx --modes process --train alexnet > gpurun_out/io_train.jsonl 2> gpurun_out/io_train.err || exit $?
cat gpurun_out/io_train.jsonl
