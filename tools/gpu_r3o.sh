#!/bin/bash
# round-3 PMC table of AlexNet b256 GEMM-shaped ops (default kernel paths)
set -o pipefail
bash tools/pmc_ops.sh r3 conv1c3_wgrad conv2_fwd conv2_dgrad conv2_wgrad conv3_fwd conv3_dgrad conv3_wgrad conv4_fwd conv5_dgrad fc6_fwd fc6_dgrad fc6_wgrad > /dev/null 2>&1 || { echo pmc failed; exit 1; }
python3 tools/pmc_table.py gpurun_out/pmcops_r3 conv1c3_wgrad conv2_fwd conv2_dgrad conv2_wgrad conv3_fwd conv3_dgrad conv3_wgrad conv4_fwd conv5_dgrad fc6_fwd fc6_dgrad fc6_wgrad > gpurun_out/pmcops_r3/table.md
bash tools/pmc_ops.sh r3r conv1c3_fwd > /dev/null 2>&1 || { echo pmc failed; exit 1; }
PMC_MATCH=rowrun python3 tools/pmc_table.py gpurun_out/pmcops_r3r conv1c3_fwd | tail -1 >> gpurun_out/pmcops_r3/table.md
cat gpurun_out/pmcops_r3/table.md
