#!/bin/bash
# Counters for probe ops at their default tiles: bash tools/pmc_ops.sh <tag> <op...>
# pass 1: issue/stall breakdown; pass 2: L2 traffic.
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcops_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for OP in "$@"; do
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/${OP}_p$i -o p -- python3 $R/benchmarks/kernel_probe.py $OP > $OUT/${OP}_p$i.log 2>&1 || { echo "pmc $OP pass $i failed"; tail -5 $OUT/${OP}_p$i.log; exit 1; }
done
python3 $R/tools/pmc_read.py $OUT/${OP}_p1 $OUT/${OP}_p2 $OUT/${OP}_p3
done
echo done
