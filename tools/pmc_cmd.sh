#!/bin/bash
# rocprofv3 PMC counters (four passes) for the kernels of one command, summarised by pmc_table.py.
#   bash tools/pmc_cmd.sh <tag> <op-name> <kernel-name-match> <program> [args...]
# e.g. bash tools/pmc_cmd.sh cd conv3_fwd conv_direct python3 benchmarks/conv_direct_probe.py --ops conv3 ...
# Counter groups respect the per-pass limits (8 SQ, 4 TCC with FETCH_SIZE = 3, 2 GRBM).
set -o pipefail
TAG=$1; OP=$2; MATCH=$3; shift 3
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TCC_HIT_sum" \
           "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/${OP}_p$i -o p -- "$@" > $OUT/${OP}_p$i.log 2>&1 || { echo "pmc $OP pass $i failed"; tail -5 $OUT/${OP}_p$i.log; exit 1; }
done
cd $R && PMC_MATCH=$MATCH python3 tools/pmc_table.py $OUT $OP | tail -1
