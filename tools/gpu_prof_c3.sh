#!/bin/bash
# Kernel-trace stats of AlexNet b256 with the 3-channel conv1 input (c3=1) and the 4-channel one (c3=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 1 0; do
  OUT=gpurun_out/prof_c3_$v
  mkdir -p $OUT
  CXXNET_CONV1_C3=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  python3 tools/prof_summary.py $OUT/prof --steps 13 --md $OUT/kernels.md > /dev/null && head -30 $OUT/kernels.md
  rm -rf $OUT/prof
done
