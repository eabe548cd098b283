#!/bin/bash
# Data-parallel step cost on one GPU: bench.py plain vs the RCCL path forced at world 1 (torchrun, dp_force=1).
set -o pipefail
OUT=gpurun_out/dpforce
mkdir -p $OUT
: > $OUT/bench.jsonl
for mb in ${MODELS:-alexnet:256 inception_v1:128 vgg16:64}; do m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 >> $OUT/bench.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
  CXXNET_DIST_FORCE=1 timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 >> $OUT/bench.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/dpforce/bench.jsonl"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(d["config"]["model"], d["ms_per_step"], d.get("dp", d["config"].get("dp")))
PY
