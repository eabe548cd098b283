#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_wgrad_halo_gpu.py > gpurun_out/r4af_test.log 2>&1 || { tail -30 gpurun_out/r4af_test.log; exit 1; }
tail -2 gpurun_out/r4af_test.log
timeout -k 10 300 python3 benchmarks/gemm_tile_probe.py --ops vgg.c1_2_wgrad,vgg.c2_2_wgrad,vgg.c3_2_wgrad,vgg.c4_2_wgrad,vgg.c5_wgrad,conv3_wgrad --tiles=-1,140,141,142 --rounds 3 --iters 5 > gpurun_out/r4af_probe.jsonl 2>&1 || exit 1
PMC_MATCH=conv_wgrad timeout -k 10 200 bash tools/pmc_tiles.sh r4af_wg vgg_c3_2_wgrad 140 || exit 1
echo done
