#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_tune_table_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tune_tests.log 2>&1
rc=$?; tail -3 $OUT/tune_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for m in "alexnet 256" "inception_v1 128" "vgg16 64"; do
  set -- $m
  timeout -k 10 300 python bench.py --model $1 --batch $2 --steps 20 --warmup 5 > $OUT/bench_$1.json 2>> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  cat $OUT/bench_$1.json
done
