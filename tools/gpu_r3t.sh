#!/bin/bash
# round-3 PMC rows for VGG-16 b64 ops and the square GEMM (the round-2 table's other rows)
set -o pipefail
bash tools/pmc_ops.sh r3v vgg_c1_2_fwd vgg_c1_2_wgrad vgg_c3_2_fwd vgg_c4_2_fwd vgg_c4_2_dgrad sq8192_fwd > /dev/null 2>&1 || { echo pmc failed; exit 1; }
python3 tools/pmc_table.py gpurun_out/pmcops_r3v vgg_c1_2_fwd vgg_c1_2_wgrad vgg_c3_2_fwd vgg_c4_2_fwd vgg_c4_2_dgrad sq8192_fwd | tee gpurun_out/pmcops_r3v/table.md
