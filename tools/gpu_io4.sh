#!/bin/bash
# Native JPEG pool (C++ threads over libjpeg-turbo, crop-window decode) on the GPU box's CPU share:
# decode alone at 8 / 16 threads against Pillow processes, then feeding AlexNet b256 training.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/io4
mkdir -p $OUT
D=/tmp/cxxnet_io_data
echo "host cpus: $(nproc), affinity: $(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
timeout -k 10 500 python -u benchmarks/io_throughput.py --dir $D --n 4096 --workers 4,8,16 --batches 16 \
    --iters imgbin,imgbinx --modes native,process > $OUT/io_decode.jsonl 2> $OUT/io_decode.err || { tail -20 $OUT/io_decode.err; exit 1; }
cut -c1-300 $OUT/io_decode.jsonl
timeout -k 10 400 python -u benchmarks/io_throughput.py --dir $D --workers 16 --batches 24 \
    --iters imgbin,imgbinx --modes native --train alexnet > $OUT/io_train.jsonl 2> $OUT/io_train.err || { tail -20 $OUT/io_train.err; exit 1; }
cut -c1-300 $OUT/io_train.jsonl
