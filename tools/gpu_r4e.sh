#!/bin/bash
# Full GPU suite + smoke + bench, then the foreign-op census of the replayed step.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_full.sh || exit $?
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 200 python -u benchmarks/foreign_ops.py --model alexnet --batch 32 > $OUT/foreign.jsonl 2> $OUT/foreign.err || tail -5 $OUT/foreign.err
cut -c1-800 $OUT/foreign.jsonl
