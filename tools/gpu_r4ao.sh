#!/bin/bash
# Shipped table with the GoogLeNet halo entries: every table entry against fp32 on the GPU, then
# the GoogLeNet and AlexNet 1-GPU benches
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4ao
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tune_table_gpu.py tests/test_conv_halo_gpu.py -q -rfE --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for m in "inception_v1 128" "alexnet 256"; do set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 20 --warmup 5 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { echo "$1 bench failed"; tail -20 $OUT/bench_$1.err; exit 1; }
  cut -c1-200 $OUT/bench_$1.json
done
