#!/bin/bash
# bench.py A/B across built worktrees under _ab/ (and the current tree), same box.
set -o pipefail
OUT=$PWD/gpurun_out/ab
mkdir -p $OUT
: > $OUT/ab.jsonl
ROOT=$PWD
for mb in ${MODELS:-alexnet:256 inception_v1:128}; do m=${mb%%:*}; b=${mb##*:}
  for d in "$@"; do
    cd $ROOT/$d || exit 1
    r=$(timeout -k 10 200 python bench.py --model $m --batch $b --steps 30 --warmup 8 2>>$OUT/ab.err | tail -1) || { tail $OUT/ab.err; exit 1; }
    echo "{\"tree\": \"$d\", \"model\": \"$m\", \"ms\": $(echo $r | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a $OUT/ab.jsonl
  done
done
