#!/bin/bash
# Same-box A/B of the 3-channel row-padded conv1 input (CXXNET_CONV1_C3=1) against the 4-channel layout.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 1 0; do
    CXXNET_CONV1_C3=$v timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > gpurun_out/ab_c3_$v.log 2>&1 || { tail -20 gpurun_out/ab_c3_$v.log; exit 1; }
    echo "c3=$v $(tail -1 gpurun_out/ab_c3_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
