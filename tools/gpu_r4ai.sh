#!/bin/bash
# Persistent halo tiles 132/133 + epilogue mask-load hoist: numerics, interleaved probe vs 130/131
# and the shipped choice, the whole GPU suite, smoke(), and an A/B of HEAD~ (_ab/base) vs this tree
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4ai
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/halo_tests.log 2>&1 || { tail -30 $OUT/halo_tests.log; exit 1; }
tail -1 $OUT/halo_tests.log
timeout -k 10 300 python -u benchmarks/gemm_tile_probe.py --ops vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_1_fwd,vgg.c2_2_fwd,vgg.c2_2_dgrad --tiles=-1,130,131,132,133 --rounds 5 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cut -c1-400 $OUT/probe.jsonl
timeout -k 10 900 python -u -m pytest tests/ -q -rfE -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -40 $OUT/tests.log | grep -E "passed|failed|FAILED|error" | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
MODELS="alexnet:256 vgg16:64" bash tools/gpu_ab_commits.sh _ab/base . _ab/base . || exit 1
cp gpurun_out/ab/ab.jsonl $OUT/ab.jsonl
