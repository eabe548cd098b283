#!/bin/bash
# Round 4: per-rank cost of the data-parallel path at AlexNet b32 (8-GPU strong-scaling share) on
# one GPU, RCCL forced at world 1: fullc_gather auto (the new default, graph-captured gathers) vs
# off, both reduction modes; plain 1-GPU step (eager and launch-list replay) for reference.
set -o pipefail
OUT=gpurun_out/dp4
mkdir -p $OUT
: > $OUT/bench.jsonl
B=${B:-32}
run() { timeout -k 10 300 python bench.py --batch $B --steps 40 --warmup 10 "$@" >> $OUT/bench.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }; }
run
CXXNET_LAUNCH_REPLAY=1 run
CXXNET_DIST_FORCE=1 run --dp-mode allreduce
CXXNET_DIST_FORCE=1 run --dp-mode shard
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --set fullc_gather=0
CXXNET_DIST_FORCE=1 run --dp-mode shard --set fullc_gather=0
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 0 --set launch_replay=1
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 0 --set launch_replay=0
python3 - <<'PY'
import json
for l in open("gpurun_out/dp4/bench.jsonl"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(d["ms_per_step"], d["dp"]["mode"], d["dp"]["fullc_gather"], d["dp"]["comm_bytes_per_step_per_rank"])
PY
