#!/bin/bash
# VGG-16 with the direct 3x3 weight-gradient: tests, in-step tuning of the cw keys, A/B vs the
# previous table (same box)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wgrad_halo_gpu.py > gpurun_out/r4ag_test.log 2>&1 || { tail -30 gpurun_out/r4ag_test.log; exit 1; }
tail -1 gpurun_out/r4ag_test.log
timeout -k 10 400 python3 benchmarks/step_tune.py --model vgg16 --batch 64 --ops cw --cands 99,140 --out gpurun_out/r4ag_vgg_cw.json > gpurun_out/r4ag_tune.log 2>&1 || { tail gpurun_out/r4ag_tune.log; exit 1; }
tail -12 gpurun_out/r4ag_tune.log
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_GEMM_TUNE_DB=tools/tbl_prev.json" "CXXNET_X=1" "CXXNET_GEMM_TUNE_DB=gpurun_out/r4ag_vgg_cw.json" "CXXNET_GEMM_TUNE_DB=tools/tbl_prev.json" "CXXNET_X=1" > gpurun_out/r4ag_ab.jsonl || exit 1
cat gpurun_out/r4ag_ab.jsonl
echo done
