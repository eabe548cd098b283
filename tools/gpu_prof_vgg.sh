#!/bin/bash
# VGG-16 kernel profile (batch 64)
set -o pipefail
OUT=gpurun_out/${1:-pv}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --model vgg16 --batch 64 --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 13 --md $OUT/kernels_vgg16.md > /dev/null && head -40 $OUT/kernels_vgg16.md
rm -f $OUT/prof/*/*kernel_trace.csv 2>/dev/null
