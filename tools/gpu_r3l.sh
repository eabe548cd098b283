#!/bin/bash
set -o pipefail
bash tools/gpu_prof_model.sh r3l_inc inception_v1 128 > /dev/null || exit 1
head -45 gpurun_out/prof_r3l_inc/kernels.md
