#!/bin/bash
# GoogLeNet: in-step tuning of conv forward / data-gradient signatures over the halo tiles, then an
# interleaved A/B of the shipped vs the tuned table (same box)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4an
mkdir -p $OUT
timeout -k 10 700 python3 -u benchmarks/step_tune.py --model inception_v1 --batch 128 --ops cf,cd --cands 130,131,133 --out $OUT/inc_tuned.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "final" $OUT/tune.log
python3 - <<'PY'
import json
a = json.load(open("cxxnet_amd/ops/glds_tune_gfx950.json")); b = json.load(open("gpurun_out/r4an/inc_tuned.json"))
for k in sorted(set(a) | set(b)):
    if a.get(k) != b.get(k): print("changed", k, a.get(k), b.get(k))
PY
bash tools/gpu_ab_env.sh inception_v1 128 "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/inc_tuned.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/inc_tuned.json" "CXXNET_X=0" "CXXNET_GEMM_TUNE_DB=$OUT/inc_tuned.json" > $OUT/ab_table.jsonl || exit 1
cat $OUT/ab_table.jsonl
