#!/bin/bash
set -o pipefail
OUT=gpurun_out/host
mkdir -p $OUT
: > $OUT/host.jsonl
for b in 32 64 256; do
  for gr in 0 1; do
    timeout -k 10 200 python benchmarks/host_overhead.py --batch $b --graph $gr >> $OUT/host.jsonl 2>> $OUT/host.err || { tail $OUT/host.err; exit 1; }
  done
done
CXXNET_DIST_FORCE=1 timeout -k 10 200 python benchmarks/host_overhead.py --batch 32 >> $OUT/host.jsonl 2>> $OUT/host.err || { tail $OUT/host.err; exit 1; }
cat $OUT/host.jsonl
