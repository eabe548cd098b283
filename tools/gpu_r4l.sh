#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4l
mkdir -p $OUT
timeout -k 10 400 python -u tools/diag_replay2.py > $OUT/d2.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/d2.log | cut -c1-3000; exit $rc
