#!/bin/bash
# conflict-free pixel assignment in the direct conv1 weight gradient: numerics, A/B vs the GEMM
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rowrun" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|^E " $OUT/t.log | head -30; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_ROWRUN_WGRAD=1" "CXXNET_ROWRUN_WGRAD=0" "CXXNET_ROWRUN_WGRAD=1" "CXXNET_ROWRUN_WGRAD=0" | tee $OUT/ab.jsonl || exit 1
CXXNET_ROWRUN_WGRAD=1 bash tools/gpu_prof_model.sh r3j_alex alexnet 256 > /dev/null || exit 1
grep -E "rowrun" gpurun_out/prof_r3j_alex/kernels.md | head; head -1 gpurun_out/prof_r3j_alex/kernels.md
