#!/bin/bash
# Data-parallel HIP-graph segments: correctness (RCCL forced world 1, gloo 2 ranks) and host overhead.
set -o pipefail
OUT=gpurun_out/dpgraph
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_dp_gpu.py \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
: > $OUT/host.jsonl
for b in 32 64 256; do
  for gr in 0 1; do
    CXXNET_DIST_FORCE=1 timeout -k 10 200 python benchmarks/host_overhead.py --batch $b --graph $gr \
        >> $OUT/host.jsonl 2>> $OUT/host.err || { tail $OUT/host.err; exit 1; }
  done
done
grep model $OUT/host.jsonl
