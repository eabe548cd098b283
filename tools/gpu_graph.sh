#!/bin/bash
# HIP-graph step: equivalence test, then eager vs graph throughput (AlexNet, GoogLeNet).
set -o pipefail
TAG=${1:-graph}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_layer_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for m in "alexnet 256" "inception_v1 128"; do
  set -- $m
  for gr in 0 1; do
    timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 30 --warmup 5 --graph $gr > $OUT/bench_$1_g$gr.json 2> $OUT/bench_$1_g$gr.err || { echo "bench $1 g$gr failed"; tail -20 $OUT/bench_$1_g$gr.err; exit 1; }
    echo "$1 graph=$gr $(cat $OUT/bench_$1_g$gr.json)"
  done
done
