#!/bin/bash
# Per-layer and per-layer-kernel GPU time for the three models (roctx ranges, trace_layers = 1).
set -o pipefail
export TMPDIR=/tmp
for spec in ${MODELS:-alexnet:256 inception_v1:128 vgg16:64}; do
  m=${spec%%:*}; b=${spec##*:}
  OUT=gpurun_out/tr3_$m
  mkdir -p $OUT
  CXXNET_TRACE_LAYERS=1 timeout -k 10 240 rocprofv3 --marker-trace --hip-trace --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --model $m --batch $b --steps 5 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  python3 tools/layer_times.py $OUT/prof --md $OUT/layers.md --kernels $OUT/layer_kernels.md | head -5
  rm -rf $OUT/prof
done
exit 0
