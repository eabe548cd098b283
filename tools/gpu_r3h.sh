#!/bin/bash
# direct row-run conv1 forward + weight-grad: numerics, AlexNet A/B, kernel profile
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rowrun or three_channel or fewc" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|^E " $OUT/t.log | head -30; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_ROWRUN_DIRECT=1" "CXXNET_ROWRUN_DIRECT=0" "CXXNET_ROWRUN_DIRECT=1" "CXXNET_ROWRUN_DIRECT=0" | tee $OUT/ab.jsonl || exit 1
bash tools/gpu_prof_model.sh r3h_alex alexnet 256 > /dev/null || exit 1
grep -E "rowrun" gpurun_out/prof_r3h_alex/kernels.md | head; head -1 gpurun_out/prof_r3h_alex/kernels.md
