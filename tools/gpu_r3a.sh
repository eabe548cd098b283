#!/bin/bash
# Round 3 session 2: zero-copy concat check, full GPU suite, 3-model bench, concat A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py -k zero_copy -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/zc.log 2>&1
rc=$?; tail -5 gpurun_out/r3a/zc.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_full.sh || exit 1
bash tools/gpu_bench3.sh || exit 1
bash tools/gpu_ab_env.sh inception_v1 128 "CXXNET_CONCAT_ZC=1" "CXXNET_CONCAT_ZC=0" "CXXNET_CONCAT_ZC=1" "CXXNET_CONCAT_ZC=0" | tee gpurun_out/r3a/ab_zc.jsonl
