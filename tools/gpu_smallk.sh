#!/bin/bash
# Kernel tests for the touched small kernels, then A/B of the three models against _ab/old.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lrn or colsum or bias or conv" > gpurun_out/smallk_tests.log 2>&1 || { tail -30 gpurun_out/smallk_tests.log; exit 1; }
tail -2 gpurun_out/smallk_tests.log
MODELS="alexnet:256 inception_v1:128 vgg16:64" bash tools/gpu_ab_commits.sh _ab/old .
