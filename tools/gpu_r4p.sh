#!/bin/bash
# Regression set after the planned-step fixes, then in-step re-tuning + benches + AlexNet profile.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r4o.sh || exit $?
bash tools/gpu_r4m.sh
