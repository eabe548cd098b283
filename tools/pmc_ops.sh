#!/bin/bash
# rocprofv3 PMC counters per GEMM op (each op in its own passes so per-kernel counters stay apart).
#   bash tools/pmc_ops.sh <tag> <probe ops...>      (ops: benchmarks/kernel_probe.py names)
# Counter groups respect the per-pass limits (8 SQ, 4 TCC with FETCH_SIZE = 3, 2 GRBM).
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcops_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for op in "$@"; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "FETCH_SIZE TCC_HIT_sum" \
             "WRITE_SIZE TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/${op}_p$i -o p -- python3 $R/benchmarks/kernel_probe.py $op > $OUT/${op}_p$i.log 2>&1 || { echo "pmc $op pass $i failed"; tail -5 $OUT/${op}_p$i.log; exit 1; }
  done
  echo "$op done"
done
python3 $R/tools/pmc_table.py $OUT "$@" > $OUT/table.md && cat $OUT/table.md
