#!/bin/bash
# Interleaved bench.py A/B of two argument sets: bash tools/gpu_ab_args.sh <tag> "<argsA>" "<argsB>" <model:batch>...
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
: > $OUT/ab.jsonl
for mb in "$@"; do m=${mb%%:*}; b=${mb##*:}
  for r in ${ROUNDS:-1 2}; do for arm in A B; do
    if [ $arm = A ]; then X="$A"; else X="$B"; fi
    timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 $X > $OUT/one.json 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
    echo "{\"arm\": \"$arm\", \"args\": \"$X\", \"model\": \"$m\", \"ms\": $(python -c "import json;print(json.loads(open('$OUT/one.json').read().strip().splitlines()[-1])['ms_per_step'])")}" | tee -a $OUT/ab.jsonl
  done; done
done
