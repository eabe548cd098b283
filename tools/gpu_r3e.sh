#!/bin/bash
# extend the shipped tile table with the signatures the current models miss (3-channel conv1 etc.)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3e
mkdir -p $OUT
CXXNET_TUNE_LOG=1 timeout -k 10 600 python -u benchmarks/tune_db.py --keep --out $OUT/glds_tune_gfx950.json \
  --models alexnet:256,alexnet:128,alexnet:64,alexnet:32,inception_v1:128,inception_v1:64,vgg16:64,vgg16:32 > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -c "not in the tile table" $OUT/tune.log; grep "not in the tile table" $OUT/tune.log | head -40
