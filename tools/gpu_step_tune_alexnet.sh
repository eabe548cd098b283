#!/bin/bash
# In-step re-tuning of AlexNet b256's tile table, then interleaved A/B of shipped vs re-tuned.
set -o pipefail
OUT=gpurun_out/st_alex
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/step_tune.py --model alexnet --batch 256 --steps 8 --rounds 2 \
  --out $OUT/table.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
tail -1 $OUT/tune.log
for i in 1 2 3; do
  for t in shipped tuned; do
    if [ $t = tuned ]; then export CXXNET_GEMM_TUNE_DB=$PWD/$OUT/table.json; else unset CXXNET_GEMM_TUNE_DB; fi
    r=$(timeout -k 10 200 python bench.py --steps 60 --warmup 15 2>>$OUT/err | tail -1) || exit 1
    echo "{\"table\": \"$t\", \"ms\": $(echo $r | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a $OUT/ab.jsonl
  done
done
