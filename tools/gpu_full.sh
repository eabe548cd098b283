#!/bin/bash
# Round-end rehearsal: the whole GPU test suite (one process), smoke(), then bench.py.
set -o pipefail
OUT=gpurun_out/full
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/ -q -rfE -m gpu --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -40 $OUT/tests.log | grep -E "passed|failed|FAILED|error" | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-220
