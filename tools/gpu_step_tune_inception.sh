#!/bin/bash
# In-step re-tuning of GoogLeNet b128's tile table (benchmarks/step_tune.py --short), then an
# interleaved A/B of the shipped vs the re-tuned table: bash tools/gpu_step_tune_inception.sh
set -o pipefail
OUT=gpurun_out/stune_inc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/step_tune.py --model inception_v1 --batch 128 --short --steps 6 --rounds 2 \
  --out $OUT/table.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
tail -2 $OUT/tune.log
