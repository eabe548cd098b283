#!/bin/bash
# Kernel profiles of AlexNet b256: plain 1-GPU step vs the data-parallel path forced at world 1.
set -o pipefail
OUT=gpurun_out/profdp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
M=${M:-alexnet}; B=${B:-256}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/plain -o run --output-format csv -- python3 bench.py --model $M --batch $B --steps 10 --warmup 3 > $OUT/plain.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/plain.log; exit 1; }
CXXNET_DIST_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dp -o run --output-format csv -- python3 bench.py --model $M --batch $B --steps 10 --warmup 3 > $OUT/dp.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/dp.log; exit 1; }
python3 tools/prof_summary.py $OUT/plain --steps 13 --md $OUT/plain.md > /dev/null && head -1 $OUT/plain.md
python3 tools/prof_summary.py $OUT/dp --steps 13 --md $OUT/dp.md > /dev/null && head -1 $OUT/dp.md
python3 tools/prof_gaps.py $OUT/plain $OUT/dp --timeline > $OUT/gaps.txt 2>&1; head -40 $OUT/gaps.txt
rm -f $OUT/*/run_kernel_trace.csv
