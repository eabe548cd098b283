#!/bin/bash
# Stall-breakdown counters of one weight-gradient arm: bash tools/pmc_wgrad.sh <tag> <layer> <arm> [batch]
set -o pipefail
TAG=$1; LAYER=$2; ARM=$3; B=${4:-256}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcwg_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p -- python3 $R/benchmarks/wgrad_probe.py --only $LAYER --arms $ARM --batch $B --rounds 2 --iters 3 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
PMC_MATCH=${PMC_MATCH:-conv_wgrad_direct<} python3 $R/tools/pmc_read.py $OUT/p1 $OUT/p2
