#!/bin/bash
# bench.py on the three model families (1 GPU), one JSON line each.
set -o pipefail
OUT=gpurun_out/bench3
mkdir -p $OUT
: > $OUT/bench.jsonl
for mb in alexnet:256 inception_v1:128 vgg16:64; do m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 >> $OUT/bench.jsonl 2>> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
done
cat $OUT/bench.jsonl
