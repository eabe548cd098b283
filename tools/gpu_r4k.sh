#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4k
mkdir -p $OUT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?
  echo "== $n rc=$rc"; grep -E "passed|failed|^FAILED|step [0-9]|single|rel |extra|Error" $OUT/$n.log | head -40
  [ $rc -le 1 ] || exit $rc
}
step rd_alex 300 python -u tools/diag_replay.py alexnet 16
step rd_alex_def 300 python -u tools/diag_replay.py alexnet 16 default
step rd_inc 300 python -u tools/diag_replay.py inception_v1 8
step dp_fp32only 200 python -u tools/diag_dp_fp32.py precision=fp32
step dp_detonly 200 python -u tools/diag_dp_fp32.py deterministic=1
step probe 500 python -u benchmarks/gemm_tile_probe.py --rounds 5 --tiles=-1,114,115,130,131 --ops vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_1_fwd,vgg.c2_2_fwd,vgg.c2_2_dgrad,vgg.c3_2_fwd,vgg.c3_2_dgrad
cut -c1-400 $OUT/probe.log
