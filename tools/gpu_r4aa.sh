#!/bin/bash
# VGG high-resolution convs: tile timings and halo-kernel PMC (conv1_2 fwd / dgrad)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 240 python3 benchmarks/gemm_tile_probe.py --ops vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_2_fwd,vgg.c2_2_dgrad --tiles=-1,130,131,113 --rounds 5 > gpurun_out/r4aa_probe.jsonl 2>&1 || exit 1
PMC_MATCH=conv_halo timeout -k 10 300 bash tools/pmc_tiles.sh r4aa_halo vgg_c1_2_fwd 130 || exit 1
cd /tmp
OUT=$R/gpurun_out/pmct_r4aa_halo
CXXNET_GLDS_TILE=130 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/t130_p3 -o p -- python3 $R/benchmarks/kernel_probe.py vgg_c1_2_fwd > $OUT/t130_p3.log 2>&1 || exit 1
cd $R && PMC_MATCH=conv_halo python3 tools/pmc_read.py $OUT/t130_p3 >> $OUT/summary.txt
echo done
