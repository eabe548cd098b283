#!/bin/bash
# Two PMC passes per (op, tile): bash tools/pmc_tiles.sh <tag> <op> <tile...>   (summary.txt)
set -o pipefail
TAG=$1; OP=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmct_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for T in "$@"; do
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    CXXNET_GLDS_TILE=$T timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/t${T}_p$i -o p -- python3 $R/benchmarks/kernel_probe.py $OP > $OUT/t${T}_p$i.log 2>&1 || { echo "pmc tile $T pass $i failed"; tail -5 $OUT/t${T}_p$i.log; exit 1; }
  done
done
cd $R
for T in "$@"; do python3 tools/pmc_read.py $OUT/t${T}_p1 $OUT/t${T}_p2; done > $OUT/summary.txt
echo done
