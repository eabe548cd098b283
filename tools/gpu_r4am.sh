#!/bin/bash
# Halo data-gradient tiles with the lower conv's bias gradient in the epilogue: numerics, then
# VGG-16 A/B with it off / on (same box), then the GEMM / halo / DP GPU tests
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4am
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/halo_tests.log 2>&1 || { tail -40 $OUT/halo_tests.log; exit 1; }
tail -1 $OUT/halo_tests.log
bash tools/gpu_ab_env.sh vgg16 64 "CXXNET_HALO_DB=0" "CXXNET_HALO_DB=1" "CXXNET_HALO_DB=0" "CXXNET_HALO_DB=1" "CXXNET_HALO_DB=0" "CXXNET_HALO_DB=1" > $OUT/ab.jsonl || exit 1
cat $OUT/ab.jsonl
timeout -k 10 900 python -u -m pytest tests/ -q -rfE -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -40 $OUT/tests.log | grep -E "passed|failed|FAILED|error" | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 240 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail $OUT/bench_default.err; exit 1; }
cut -c1-200 $OUT/bench_default.json
exit $rc
