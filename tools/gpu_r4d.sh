#!/bin/bash
# Re-entry check of round 4's new code on a fresh box: new-tile numerics + probe, launch-list
# executor, host cost; then the whole GPU suite, smoke and bench.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r4c.sh || exit $?
bash tools/gpu_full.sh
