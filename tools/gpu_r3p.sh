#!/bin/bash
# 256x192 / 192x256 tiles: numerics on the candidate shapes, then AlexNet in-step re-tune of cf / cd
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tune_table_gpu.py -k "every_candidate_tile and (82 or 83)" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "PASS|FAIL|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u benchmarks/step_tune.py --model alexnet --batch 256 --ops cf,cd --rounds 3 --out $OUT/table.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
cut -c1-200 $OUT/tune.log
