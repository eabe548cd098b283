#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2d/kt.log 2>&1
rc=$?; tail -3 gpurun_out/r2d/kt.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python benchmarks/gemm_glds_bench.py --iters 20 --ops conv2_wgrad,conv3_wgrad,conv4_wgrad,conv5_wgrad,conv1_wgrad,fc6_wgrad,fc7_wgrad,vgg.c3_2_wgrad,vgg.c4_2_wgrad --tiles 1,17,23,36,40,41 > gpurun_out/r2d/sweep_wgrad.jsonl 2> gpurun_out/r2d/sweep.err || { tail gpurun_out/r2d/sweep.err; exit 1; }
cat gpurun_out/r2d/sweep_wgrad.jsonl
