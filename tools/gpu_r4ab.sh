#!/bin/bash
# VGG weight-gradient: tile timings (table / LDS-DMA MN tiles / tile 120) and register-kernel PMC
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python3 benchmarks/gemm_tile_probe.py --ops vgg.c1_2_wgrad,vgg.c2_2_wgrad,vgg.c3_2_wgrad,vgg.c4_2_wgrad,vgg.c5_wgrad --tiles=-1,1,2,13,17,23,36,40,41,120 --rounds 3 --iters 5 > gpurun_out/r4ab_probe.jsonl 2>&1 || exit 1
PMC_MATCH=gemm_kernel timeout -k 10 200 bash tools/pmc_tiles.sh r4ab_reg vgg_c3_2_wgrad -1 || exit 1
PMC_MATCH=gemm_kernel timeout -k 10 200 bash tools/pmc_tiles.sh r4ab_reg1 vgg_c1_2_wgrad -1 || exit 1
echo done
