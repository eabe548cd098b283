#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_e2e_gpu.py -x -q -s --timeout 600 --timeout-method thread -k trajectory > $OUT/traj.log 2>&1
rc=$?; tail -12 $OUT/traj.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tie or rows_even" > $OUT/k.log 2>&1
rc=$?; tail -3 $OUT/k.log; exit $rc
