#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_full.sh || exit $?
bash tools/gpu_r4w.sh
