#!/bin/bash
# Tile-table correctness gate + forced single-rank RCCL bench (DP machinery on one GPU).
set -o pipefail
OUT=gpurun_out/r2b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_tune_table_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tune_tests.log 2>&1
rc=$?; echo "tune tests rc=$rc"; tail -5 $OUT/tune_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
CXXNET_DIST_FORCE=1 timeout -k 10 180 python bench.py --steps 30 --warmup 10 > $OUT/bench_force_shard.json 2> $OUT/bench_force.err || { echo "bench failed"; tail -20 $OUT/bench_force.err; exit 1; }
cat $OUT/bench_force_shard.json
CXXNET_DIST_FORCE=1 timeout -k 10 180 python bench.py --steps 30 --warmup 10 --dp-mode allreduce > $OUT/bench_force_ar.json 2>> $OUT/bench_force.err || { echo "bench failed"; tail -20 $OUT/bench_force.err; exit 1; }
cat $OUT/bench_force_ar.json
timeout -k 10 180 python bench.py --steps 30 --warmup 10 --scaling strong --batch 32 > $OUT/bench_b32.json 2>> $OUT/bench_force.err || { echo "bench failed"; tail -20 $OUT/bench_force.err; exit 1; }
cat $OUT/bench_b32.json
