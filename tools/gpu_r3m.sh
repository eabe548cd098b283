#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r3m
mkdir -p $OUT
CXXNET_DIST_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --batch 32 --steps 10 --warmup 3 --dp-mode allreduce > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r3m/prof/**/*kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/r3m/prof/*kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    n = r.get("Name") or r.get("KernelName") or ""
    if "transpose" in n.lower() or "rocclr" in n.lower() or "nccl" in n.lower() or "elementwise" in n.lower():
        print(r.get("Calls"), r.get("TotalDurationNs"), n[:300])
PY
