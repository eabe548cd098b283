#!/bin/bash
# One GPU verification round: gpu tests, bench, kernel profile.  Usage (on the box):
#   bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/tests.log
# 0 = pass, 1 = test failures; anything else (abort/segv/timeout) ends the call
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/$TAG/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/prof -o run -- python bench.py --steps 10 --warmup 3 "$@" > gpurun_out/$TAG/prof.log 2>&1 || { echo prof failed; tail -5 gpurun_out/$TAG/prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/$TAG/prof --steps 13 --md gpurun_out/$TAG/kernels.md > /dev/null && head -1 gpurun_out/$TAG/kernels.md
rm -rf gpurun_out/$TAG/prof/*/*.csv.tmp 2>/dev/null
exit 0
