#!/bin/bash
# conv1 forward: round-4 rework vs round-3 form, timing + PMC (bank conflicts, VALU, MFMA busy)
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4u
mkdir -p $OUT
timeout -k 10 120 python -u benchmarks/conv1_time.py --arms new,r3 --rounds 9 2>&1 | grep op
cd /tmp
for arm in new r3; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/$arm -o p -- python3 $GRAFT_REPO_ROOT/benchmarks/conv1_time.py --arms $arm --rounds 2 --iters 3 > $OUT/$arm.log 2>&1 || { echo "pmc $arm failed"; tail -3 $OUT/$arm.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for arm in new r3; do PMC_MATCH=rowrun python3 tools/pmc_read.py $OUT/$arm; done
