#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4r
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -q -k rowrun --timeout 60 --timeout-method thread -p no:cacheprovider > $OUT/rr.log 2>&1; echo "rowrun tests rc=$?"; tail -1 $OUT/rr.log
timeout -k 10 120 python -u benchmarks/conv1_time.py > $OUT/conv1.jsonl 2>&1; echo "conv1 rc=$?"; grep op $OUT/conv1.jsonl
timeout -k 10 300 python -u tools/diag_e2e.py > $OUT/e2e.log 2>&1; echo "diag rc=$?"; grep -v amdgpu $OUT/e2e.log | head -40
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_launch_hygiene_gpu.py -q -rfE --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|^FAILED" $OUT/t.log
timeout -k 10 600 bash tools/gpu_dp4.sh || exit $?
timeout -k 10 500 bash tools/gpu_io4.sh
bash tools/pmc_tiles.sh r4sq sq8192_fwd 21 110 113 && cat gpurun_out/pmct_r4sq/summary.txt
