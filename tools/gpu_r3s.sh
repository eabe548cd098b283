#!/bin/bash
# fused fc SGD on a side stream: bitwise test, then AlexNet / VGG-16 A/B
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_sgd_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "PASS|FAIL|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_FC_SGD_SIDE=1" "CXXNET_FC_SGD_SIDE=0" "CXXNET_FC_SGD_SIDE=1" "CXXNET_FC_SGD_SIDE=0" "CXXNET_FC_SGD_SIDE=1" "CXXNET_FC_SGD_SIDE=0" | tee $OUT/ab_alex.jsonl || exit 1
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_FC_SGD_SIDE=1" "CXXNET_FC_SGD_SIDE=0" "CXXNET_FC_SGD_SIDE=1" "CXXNET_FC_SGD_SIDE=0" | tee $OUT/ab_vgg.jsonl || exit 1
