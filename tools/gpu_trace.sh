#!/bin/bash
# Per-layer GPU time (default AlexNet b256; args: tag model batch): roctx range per layer (trace_layers = 1) + HIP API + kernel trace.
set -o pipefail
OUT=gpurun_out/${1:-tr}
mkdir -p $OUT
export TMPDIR=/tmp
CXXNET_TRACE_LAYERS=1 timeout -k 10 240 rocprofv3 --marker-trace --hip-trace --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --model ${2:-alexnet} --batch ${3:-256} --steps 5 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/layer_times.py $OUT/prof --md $OUT/layers.md | head -60
rm -f $OUT/prof/*/*hip_api_trace.csv $OUT/prof/*hip_api_trace.csv 2>/dev/null
exit 0
