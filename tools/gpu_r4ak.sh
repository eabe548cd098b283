#!/bin/bash
# Round-4 close-out on HEAD: whole GPU suite, smoke(), 1-GPU benches of the three models, VGG-16
# and AlexNet kernel traces
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4ak
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -q -rfE -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -40 $OUT/tests.log | grep -E "passed|failed|FAILED|error" | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for m in "alexnet 256" "vgg16 64" "inception_v1 128"; do set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --batch $2 --steps 20 --warmup 5 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { echo "$1 bench failed"; tail -20 $OUT/bench_$1.err; exit 1; }
  cut -c1-200 $OUT/bench_$1.json
done
timeout -k 10 240 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail $OUT/bench_default.err; exit 1; }
cut -c1-200 $OUT/bench_default.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_vgg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model vgg16 --batch 64 --steps 8 --warmup 4 > $GRAFT_REPO_ROOT/$OUT/prof_vgg.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$OUT/prof_vgg.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/prof_summary.py $OUT/prof_vgg --steps 12 --md $OUT/kernels_vgg.md > /dev/null && head -14 $OUT/kernels_vgg.md
