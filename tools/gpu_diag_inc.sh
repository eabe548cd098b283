#!/bin/bash
# GoogLeNet b128 step time under tuning on/off, then a kernel profile of the default run.
set -o pipefail
OUT=gpurun_out/diag_inc
mkdir -p $OUT
: > $OUT/bench.jsonl
for env in "X=1" "CXXNET_GEMM_TUNE=0" "X=2"; do
  env $env timeout -k 10 300 python bench.py --model inception_v1 --batch 128 --steps 30 --warmup 8 >> $OUT/bench.jsonl 2>> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  echo "$env $(tail -1 $OUT/bench.jsonl | cut -c1-200)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --model inception_v1 --batch 128 --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 13 --md $OUT/kernels.md > /dev/null && head -30 $OUT/kernels.md
