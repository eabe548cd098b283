#!/bin/bash
# conv1 c3 leak fix check, fc GEMMs vs hipBLASLt, AlexNet b256 kernel profile
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_fused_sgd_gpu.py tests/test_kernels_gpu.py -k "fused_fc_sgd or three_channel" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/c3.log 2>&1; rc=$?; grep -E "PASS|FAIL" $OUT/c3.log | head -20; tail -2 $OUT/c3.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u benchmarks/fc_lib_probe.py > $OUT/fc_lib.jsonl 2>$OUT/fc.err || { tail $OUT/fc.err; exit 1; }
cat $OUT/fc_lib.jsonl
bash tools/gpu_prof_model.sh r3d_alex alexnet 256
