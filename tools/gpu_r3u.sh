#!/bin/bash
# conv1 direct forward with fixed-count buffer stores (epilogue stores drain behind the next item)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "rowrun or three_channel" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof_model.sh r3u_alex alexnet 256 > /dev/null || exit 1
grep -E "rowrun" gpurun_out/prof_r3u_alex/kernels.md | head -3; head -1 gpurun_out/prof_r3u_alex/kernels.md
timeout -k 10 200 python bench.py > $OUT/bench.json 2>$OUT/bench.err || exit 1
cut -c1-160 $OUT/bench.json
