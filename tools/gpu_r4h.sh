#!/bin/bash
# Round-4 regression fix check: the previously failing GPU tests with the plan invalidation /
# workspace retirement fixes; if any still fail, the same set with the launch-list executor off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4h
mkdir -p $OUT
T="tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py tests/test_fused_sgd_gpu.py tests/test_launch_replay_gpu.py tests/test_kernels_gpu.py"
timeout -k 10 560 python -u -m pytest $T -q -rfE -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t1.log 2>&1; rc=$?
echo "fixed rc=$rc"; grep -E "passed|failed|^FAILED|err " $OUT/t1.log | head -40
[ $rc -le 1 ] || exit $rc
if [ $rc -eq 1 ]; then
  CXXNET_LAUNCH_REPLAY=0 timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py -q -rfE -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t0.log 2>&1
  echo "replay off rc=$?"; grep -E "passed|failed|^FAILED|err " $OUT/t0.log | head -30
fi
