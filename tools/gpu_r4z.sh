#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_prof_model.sh r4z_alex alexnet 256 || exit 1
bash tools/gpu_prof_model.sh r4z_vgg vgg16 64 || exit 1
