#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3r
bash tools/gpu_ab_env.sh alexnet 256 "CXXNET_GEMM_TUNE_DB=benchmarks/tables/r3_before_82.json" "CXXNET_X=1" "CXXNET_GEMM_TUNE_DB=benchmarks/tables/r3_before_82.json" "CXXNET_X=1" "CXXNET_GEMM_TUNE_DB=benchmarks/tables/r3_before_82.json" "CXXNET_X=1" | tee gpurun_out/r3r/ab.jsonl
