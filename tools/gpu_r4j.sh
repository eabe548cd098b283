#!/bin/bash
# Replay fix (library-memset gradient zeroing), halo conv kernel, conflict-free conv1 forward.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4j
mkdir -p $OUT
step() {  # name, timeout, command...: test failures (rc 1) continue, crashes / timeouts stop
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc"; grep -E "passed|failed|^FAILED|step [0-9]|single" $OUT/$n.log | head -30
  [ $rc -le 1 ] || exit $rc
}
step halo 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q -rfE --timeout 120 --timeout-method thread -p no:cacheprovider
step replaydiag 200 python -u tools/diag_replay.py small 8
step regress 500 python -u -m pytest tests/test_determinism_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py tests/test_fused_sgd_gpu.py tests/test_launch_replay_gpu.py -q -rfE --timeout 150 --timeout-method thread -p no:cacheprovider
step kern 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_4w_gpu.py -q -rfE --timeout 120 --timeout-method thread -p no:cacheprovider
step dpfp32 200 python -u tools/diag_dp_fp32.py
step probe 500 python -u benchmarks/gemm_tile_probe.py --rounds 5 --tiles -1,114,115,130,131 --ops vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_1_fwd,vgg.c2_2_fwd,vgg.c2_2_dgrad,vgg.c3_2_fwd,vgg.c3_2_dgrad
cut -c1-400 $OUT/probe.log
