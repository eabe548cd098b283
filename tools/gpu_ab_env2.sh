#!/bin/bash
# Interleaved bench.py A/B of an env toggle: bash tools/gpu_ab_env2.sh <tag> "<envA>" "<envB>" <model:batch>...
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
: > $OUT/ab.jsonl
for mb in "$@"; do m=${mb%%:*}; b=${mb##*:}
  for r in ${ROUNDS:-1 2}; do for arm in A B; do
    if [ $arm = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 > $OUT/one.json 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
    echo "{\"arm\": \"$arm\", \"env\": \"$E\", \"model\": \"$m\", \"ms\": $(python -c "import json;print(json.loads(open('$OUT/one.json').read().strip().splitlines()[-1])['ms_per_step'])")}" | tee -a $OUT/ab.jsonl
  done; done
done
