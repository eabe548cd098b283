#!/bin/bash
# One GPU round trip: GPU tests, smoke, 1-GPU bench, and a rocprofv3 kernel-trace summary.
#   bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 180 python bench.py --steps 30 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 13 --warmup 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 18 --md $OUT/kernels.md > /dev/null && head -3 $OUT/kernels.md
