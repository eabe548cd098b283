#!/bin/bash
# Host enqueue cost vs GPU time per step (benchmarks/host_overhead.py), plain and data-parallel
# (RCCL forced at world 1), AlexNet b32 / b256, launch lists (default) and HIP graphs.
#   bash tools/gpu_host_overhead.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-host}
mkdir -p $OUT
export TMPDIR=/tmp
for b in 32 256; do
  for g in -1 1; do
    timeout -k 10 200 python -u benchmarks/host_overhead.py --batch $b --graph $g --steps 10 >> $OUT/host.jsonl 2>> $OUT/host.err || { echo "plain b$b g$g failed"; tail -5 $OUT/host.err; exit 1; }
    CXXNET_DIST_FORCE=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29731 benchmarks/host_overhead.py --batch $b --graph $g --steps 10 >> $OUT/host_dp.jsonl 2>> $OUT/host.err || { echo "dp b$b g$g failed"; tail -5 $OUT/host.err; exit 1; }
  done
done
cat $OUT/host.jsonl $OUT/host_dp.jsonl
