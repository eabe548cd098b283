#!/bin/bash
# Strong-scaling per-rank cost at AlexNet b32 (RCCL forced at world 1): graph segments vs launch
# lists, with and without fullc_gather; kernel traces of the plain and the best DP step.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4w
mkdir -p $OUT
: > $OUT/bench.jsonl
run() { timeout -k 10 300 python bench.py --batch 32 --steps 40 --warmup 10 "$@" >> $OUT/bench.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }; }
run
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 1
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 0 --set launch_replay=1
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 1 --set fullc_gather=0
CXXNET_DIST_FORCE=1 run --dp-mode allreduce --graph 0 --set launch_replay=1 --set fullc_gather=0
python3 - <<'PY'
import json
for l in open("gpurun_out/r4w/bench.jsonl"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(d["ms_per_step"], d["dp"]["mode"], d["dp"]["fullc_gather"], d["dp"]["comm_bytes_per_step_per_rank"])
PY
cd /tmp
for v in plain dp; do
  if [ $v = plain ]; then E=""; A=""; else E="CXXNET_DIST_FORCE=1"; A="--dp-mode allreduce --graph 0 --set launch_replay=1"; fi
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 32 --steps 20 --warmup 5 $A > $GRAFT_REPO_ROOT/$OUT/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $GRAFT_REPO_ROOT/$OUT/prof_$v.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for v in plain dp; do python3 tools/prof_summary.py $OUT/prof_$v --steps 25 --md $OUT/kernels_$v.md > /dev/null; head -28 $OUT/kernels_$v.md | cut -c1-160; done
