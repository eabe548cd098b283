#!/bin/bash
# Tile-table correctness gate, then the three model benches.
set -o pipefail
OUT=gpurun_out/table
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tune_table_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_bench3.sh
