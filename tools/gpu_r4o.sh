#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4o
mkdir -p $OUT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc"; grep -E "passed|failed|^FAILED|step [0-9]|^   |AssertionError" $OUT/$n.log | cut -c1-600 | head -40
  [ $rc -le 1 ] || exit $rc
}
step plans 400 python -u tools/diag_plans.py alexnet 16
step regress 600 python -u -m pytest tests/test_dp_gpu.py tests/test_e2e_gpu.py tests/test_fused_sgd_gpu.py tests/test_launch_replay_gpu.py tests/test_launch_hygiene_gpu.py tests/test_determinism_gpu.py -q -rfE --timeout 150 --timeout-method thread -p no:cacheprovider
