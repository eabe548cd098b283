#!/bin/bash
# direct row-run conv1 forward: numerics, then AlexNet A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rowrun or three_channel" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "PASS|FAIL|^E " $OUT/t.log | head -30; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_ROWRUN_DIRECT=1" "CXXNET_ROWRUN_DIRECT=0" "CXXNET_ROWRUN_DIRECT=1" "CXXNET_ROWRUN_DIRECT=0" | tee $OUT/ab.jsonl || exit 1
bash tools/gpu_prof_model.sh r3g_alex alexnet 256 > /dev/null || exit 1
grep -E "rowrun|K_ROW|96, 128, 2, 2, 2, 0, 4" gpurun_out/prof_r3g_alex/kernels.md | head; head -1 gpurun_out/prof_r3g_alex/kernels.md
# few-channel first-layer forward kernel A/B on GoogLeNet and VGG-16, then the AlexNet kernel profile
mkdir -p gpurun_out/r3f
bash tools/gpu_ab_env.sh inception_v1 128 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3f/ab_fewc_inc.jsonl || exit 1
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3f/ab_fewc_vgg.jsonl || exit 1
