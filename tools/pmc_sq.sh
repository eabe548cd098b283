#!/bin/bash
# PMC passes for square GEMMs: hipBLASLt (torch.mm) and our tiles.  bash tools/pmc_sq.sh <tag> <n> <tile...>
set -o pipefail
TAG=$1; N=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcsq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/blas_p$i -o p -- python3 $R/benchmarks/blas_probe.py $N > $OUT/blas_p$i.log 2>&1 || { echo "pmc blas pass $i failed"; tail -5 $OUT/blas_p$i.log; exit 1; }
  for T in "$@"; do
    CXXNET_GLDS_TILE=$T timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/t${T}_p$i -o p -- python3 $R/benchmarks/kernel_probe.py sq${N}_fwd > $OUT/t${T}_p$i.log 2>&1 || { echo "pmc tile $T pass $i failed"; tail -5 $OUT/t${T}_p$i.log; exit 1; }
  done
done
cd $R
for d in $OUT/*_p1; do
  b=${d%_p1}; m=gemm; case $b in *blas) m=Cijk;; esac
  PMC_MATCH=$m python3 tools/pmc_read.py ${b}_p1 ${b}_p2
done > $OUT/summary.txt
grep -h "Kernel_Name" -A0 $OUT/blas_p1/*/*kernel_trace.csv > /dev/null 2>&1
python3 - "$OUT" <<'PY' >> $OUT/summary.txt
import csv, glob, sys
names = set()
for p in glob.glob(sys.argv[1] + "/blas_p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "Cijk" in r["Kernel_Name"]:
            names.add((r["Kernel_Name"], r.get("VGPR_Count", "?"), r.get("Accum_VGPR_Count", "?"), r.get("LDS_Block_Size", r.get("Lds_Size", "?")), r.get("Workgroup_Size", "?")))
for n in names:
    print("BLAS kernel:", n)
PY
echo done
