#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4s
mkdir -p $OUT
for v in "DIAG_EAGER=1" "DIAG_EAGER=1 CXXNET_FUSE_FC_SGD=0" "DIAG_EAGER=0"; do
  echo "== $v"
  env $v timeout -k 10 200 python -u tools/diag_e2e.py 2>&1 | grep -v amdgpu | cut -c1-300 | head -24
done
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/pmc_c1 -o p -- python3 benchmarks/conv1_time.py --rounds 2 --iters 3 > $OUT/pmc_c1.log 2>&1; echo "pmc rc=$?"
python3 tools/pmc_read.py $OUT/pmc_c1 2>&1 | head -20
