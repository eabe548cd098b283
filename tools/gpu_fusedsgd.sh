#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_fused_sgd_gpu.py tests/test_e2e_gpu.py tests/test_dp_gpu.py > gpurun_out/fsgd_tests.log 2>&1 || { tail -40 gpurun_out/fsgd_tests.log; exit 1; }
tail -3 gpurun_out/fsgd_tests.log
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_FUSE_FC_SGD=0" "CXXNET_FUSE_FC_SGD=1" "CXXNET_FUSE_FC_SGD=0" "CXXNET_FUSE_FC_SGD=1"
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_FUSE_FC_SGD=0" "CXXNET_FUSE_FC_SGD=1"
