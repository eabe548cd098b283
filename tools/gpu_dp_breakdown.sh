#!/bin/bash
# Per-rank cost of the data-parallel path at AlexNet b32 (the 8-GPU strong-scaling share) on one
# GPU: plain step vs the RCCL path forced at world 1 in each reduction mode, plus a kernel trace of
# the forced all-reduce step that separates RCCL's own kernels (its world-1 local copies).
set -o pipefail
OUT=gpurun_out/dpbd
mkdir -p $OUT
: > $OUT/bench.jsonl
B=${B:-32}
run() { timeout -k 10 300 python bench.py --batch $B --steps 40 --warmup 10 "$@" >> $OUT/bench.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }; }
run
CXXNET_DIST_FORCE=1 run --dp-mode allreduce
CXXNET_DIST_FORCE=1 run --dp-mode shard
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --set fullc_gather=1
CXXNET_DIST_FORCE=1 run --dp-mode shard --set fullc_gather=1
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CXXNET_DIST_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_ar -o run -- python3 bench.py --batch $B --steps 10 --warmup 3 --dp-mode allreduce > $OUT/prof_ar.log 2>&1 || { tail $OUT/prof_ar.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_plain -o run -- python3 bench.py --batch $B --steps 10 --warmup 3 > $OUT/prof_plain.log 2>&1 || { tail $OUT/prof_plain.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof_ar --steps 13 --md $OUT/kernels_ar.md > /dev/null
python3 tools/prof_summary.py $OUT/prof_plain --steps 13 --md $OUT/kernels_plain.md > /dev/null
python3 - <<'PY'
import json
for l in open("gpurun_out/dpbd/bench.jsonl"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(d["ms_per_step"], d["dp"])
PY
