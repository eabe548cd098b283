#!/bin/bash
# rocprofv3 PMC counters for the top GEMM kernels of AlexNet / VGG-16 (one counter group per pass).
#   bash tools/pmc_top.sh <tag> <probe ops...>
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TCC_HIT_sum TCC_MISS_sum" \
           "WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $R/benchmarks/kernel_probe.py "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc done
