#!/bin/bash
# Round-4 baseline on a fresh box: full GPU suite + smoke + AlexNet bench, then GoogLeNet / VGG-16 benches.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_full.sh || exit $?
OUT=gpurun_out/r4a
mkdir -p $OUT
for m in "inception_v1 128" "vgg16 64" "alexnet 256"; do
  set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 20 --warmup 5 >> $OUT/bench_models.jsonl 2> $OUT/bench_$1.err || { echo "$1 bench failed"; tail -20 $OUT/bench_$1.err; exit 1; }
done
cut -c1-200 $OUT/bench_models.jsonl
