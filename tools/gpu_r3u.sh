#!/bin/bash
# conv1 direct forward with fixed-count buffer stores: numerics (incl. 40-image multi-item case),
# A/B counted wait vs vmcnt(0), then the full suite + smoke + bench
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rowrun or three_channel" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_ROWRUN_COUNTED=1" "CXXNET_ROWRUN_COUNTED=0" "CXXNET_ROWRUN_COUNTED=1" "CXXNET_ROWRUN_COUNTED=0" | tee $OUT/ab.jsonl || exit 1
bash tools/gpu_full.sh
