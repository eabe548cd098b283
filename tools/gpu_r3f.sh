#!/bin/bash
# few-channel first-layer forward kernel A/B on GoogLeNet and VGG-16, then the AlexNet kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3f
bash tools/gpu_ab_env.sh inception_v1 128 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3f/ab_fewc_inc.jsonl || exit 1
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_FEWC=1" "CXXNET_FEWC=0" "CXXNET_FEWC=1" "CXXNET_FEWC=0" | tee gpurun_out/r3f/ab_fewc_vgg.jsonl || exit 1
bash tools/gpu_prof_model.sh r3f_alex alexnet 256 > /dev/null || exit 1
head -3 gpurun_out/prof_r3f_alex/kernels.md
