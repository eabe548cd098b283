#!/bin/bash
# 256x192 / 192x256 tiles on the other models' conv forward / data-grad signatures (in-step)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3q
mkdir -p $OUT
for m in "vgg16 64" "inception_v1 128" "alexnet 32" "alexnet 64" "alexnet 128"; do
  set -- $m
  timeout -k 10 900 python -u benchmarks/step_tune.py --model $1 --batch $2 --ops cf,cd --cands 82,83 --rounds 3 --out $OUT/table_$1_$2.json > $OUT/tune_$1_$2.log 2>&1 || { tail -20 $OUT/tune_$1_$2.log; exit 1; }
  grep -v '"old": \([0-9]*\), "old_ms": [0-9.]*, "new": \1,' $OUT/tune_$1_$2.log | cut -c1-200
done
