#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_determinism_gpu.py tests/test_metrics_gpu.py -x -q --timeout 120 --timeout-method thread -k "metric or bitwise or deterministic" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -m cxxnet_amd cxxnet_amd/models/confs/alexnet.conf max_round=3 num_round=3 save_model=0 profile_step=1 print_step=50 synthetic_dtype=uint8 model_dir=/tmp/cxm > $OUT/cli_alexnet.log 2>&1 || { tail -20 $OUT/cli_alexnet.log; exit 1; }
cat $OUT/cli_alexnet.log | tr '\r' '\n' | grep -v "^ *$" | tail -12
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
