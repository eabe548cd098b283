#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 200 python -u tools/diag_replay.py small 8 2>&1 | tee $OUT/small.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/diag_replay.py alexnet 16 2>&1 | tee $OUT/alexnet.log | grep -v amdgpu.ids
