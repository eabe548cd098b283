#!/bin/bash
# In-step re-tuning with the round-4 tiles as candidates (one-wave-per-SIMD 110-115, halo conv
# 130-131), chained over the models, then the three benches on the new table.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tune4
mkdir -p $OUT
T=cxxnet_amd/ops/glds_tune_gfx950.json
run() {  # name in_table out_table args...
  local n=$1 tin=$2 tout=$3; shift 3
  CXXNET_GEMM_TUNE_DB=$tin timeout -k 10 420 python -u benchmarks/step_tune.py --out $tout "$@" > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  grep -c '"new"' $OUT/$n.log; python3 -c "
import json
ch=[json.loads(l) for l in open('$OUT/$n.log') if l.startswith('{')]
ch=[c for c in ch if c['new']!=c['old']]
print('$n changed', len(ch)); [print(' ', c) for c in ch]"; grep final $OUT/$n.log
}
run alex256 $T $OUT/t1.json --model alexnet --batch 256 --ops cf,cd,fc --cands 110,111,112,113,114,115
run alex32 $OUT/t1.json $OUT/t2.json --model alexnet --batch 32 --ops cf,cd,fc --cands 110,111,112,113,114,115
run vgg64 $OUT/t2.json $OUT/t3.json --model vgg16 --batch 64 --ops cf,cd,fc --cands 110,111,112,113,114,115,130,131
run inc128 $OUT/t3.json $OUT/t4.json --model inception_v1 --batch 128 --ops cf,cd --cands 110,112,114,115
for m in "alexnet 256" "vgg16 64" "inception_v1 128"; do
  set -- $m
  CXXNET_GEMM_TUNE_DB=$OUT/t4.json timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 20 --warmup 5 >> $OUT/bench.jsonl 2> $OUT/bench_$1.err || { echo "$1 bench failed"; tail -5 $OUT/bench_$1.err; exit 1; }
done
cut -c1-200 $OUT/bench.jsonl
export CXXNET_GEMM_TUNE_DB=$OUT/t4.json
bash tools/gpu_prof_model.sh r4alex alexnet 256 || exit 1
