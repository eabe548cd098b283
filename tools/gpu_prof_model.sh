#!/bin/bash
# Kernel-trace profile of one model's training step.  bash tools/gpu_prof_model.sh <tag> <model> <batch>
set -o pipefail
TAG=$1; M=$2; B=$3
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --model $M --batch $B --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 13 --md $OUT/kernels.md > /dev/null && head -40 $OUT/kernels.md
