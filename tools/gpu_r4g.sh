#!/bin/bash
# Bisect the round-4 GPU test regressions: the failing tests with the launch-list executor off.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4g
mkdir -p $OUT
CXXNET_LAUNCH_REPLAY=0 timeout -k 10 500 python -u -m pytest tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py tests/test_fused_sgd_gpu.py -q -rfE -s --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t0.log 2>&1; echo "replay off rc=$?"
grep -E "passed|failed|^FAILED|err " $OUT/t0.log | head -40
