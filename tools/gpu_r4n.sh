#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4n
mkdir -p $OUT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc"; grep -E "passed|failed|^FAILED|step [0-9]|replay=" $OUT/$n.log | cut -c1-400 | head -30
  [ $rc -le 1 ] || exit $rc
}
step d2 300 python -u tools/diag_replay2.py
step regress 500 python -u -m pytest tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py tests/test_fused_sgd_gpu.py tests/test_launch_replay_gpu.py tests/test_kernels_gpu.py -q -rfE --timeout 150 --timeout-method thread -p no:cacheprovider
