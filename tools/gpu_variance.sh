#!/bin/bash
# Repeated fresh-process GoogLeNet / AlexNet benches with table-miss logging (bimodal step times?).
set -o pipefail
OUT=gpurun_out/variance
mkdir -p $OUT
: > $OUT/runs.jsonl
for r in 1 2 3 4 5; do for mb in inception_v1:128 alexnet:256; do m=${mb%%:*}; b=${mb##*:}
  CXXNET_TUNE_LOG=1 timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 8 > $OUT/one.json 2> $OUT/err_${m}_$r.log || { tail $OUT/err_${m}_$r.log; exit 1; }
  echo "{\"run\": $r, \"model\": \"$m\", \"ms\": $(python -c "import json;print(json.loads(open('$OUT/one.json').read().strip().splitlines()[-1])['ms_per_step'])"), \"misses\": $(grep -c 'gemm tune' $OUT/err_${m}_$r.log)}" | tee -a $OUT/runs.jsonl
done; done
