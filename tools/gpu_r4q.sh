#!/bin/bash
# Strong-scaling per-rank cost at AlexNet b32 (RCCL forced at world 1) and the native JPEG pool.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_dp4.sh || exit $?
timeout -k 10 500 bash tools/gpu_io4.sh
