#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
PYTHONPATH=. timeout -k 10 150 python -u tools/diag_conv1c3.py > gpurun_out/r3c/diag_c3.log 2>&1; rc=$?; cat gpurun_out/r3c/diag_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "three_channel or row_padded" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c/c3.log 2>&1; grep -E "PASS|FAIL|Error|assert" gpurun_out/r3c/c3.log | head -40; tail -3 gpurun_out/r3c/c3.log
