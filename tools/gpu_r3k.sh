#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_tune_table_gpu.py -k "cwr or cr" -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; tail -3 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
for m in "alexnet 256" "inception_v1 128" "vgg16 64"; do
  set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 30 --warmup 8 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { tail $OUT/bench_$1.err; exit 1; }
  cut -c1-200 $OUT/bench_$1.json
done
