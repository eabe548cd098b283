#!/bin/bash
# Kernel-trace profiles of one model in two trees (same box): bash tools/gpu_ab_prof.sh <model> <batch> <treeA> <treeB>
set -o pipefail
M=$1; B=$2; shift 2
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp && cd $ROOT
for d in "$@"; do
  tag=$(echo $d | tr '/.' '__')
  OUT=$ROOT/gpurun_out/abprof/$tag
  mkdir -p $OUT
  cd $ROOT/$d || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --model $M --batch $B --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  cd $ROOT
  python3 tools/prof_summary.py $OUT/prof --steps 13 --md $OUT/kernels.md > /dev/null && head -30 $OUT/kernels.md
done
