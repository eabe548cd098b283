#!/bin/bash
# in-step re-tuning of AlexNet b256's tile table entries (after the conv1 input / kernel changes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3n
mkdir -p $OUT
timeout -k 10 900 python -u benchmarks/step_tune.py --model alexnet --batch 256 --out $OUT/table.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -v '"old": \([0-9]*\), "old_ms": [0-9.]*, "new": \1,' $OUT/tune.log | tail -30
