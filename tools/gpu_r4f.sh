#!/bin/bash
# Conflict-free conv1 forward (tests + timing), 4w tiles against the shipped table's choices on
# AlexNet / VGG shapes, then in-step re-tuning of AlexNet b256 with the 4w tiles as candidates.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_4w_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1; rc=$?; grep -E "FAIL|Error|^E " $OUT/t.log | head -20; tail -2 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u benchmarks/gemm_tile_probe.py --rounds 5 --tiles -1,110,112,113,114,115 \
  --ops conv1_fwd,conv2_dgrad,conv3_fwd,conv3_dgrad,conv4_fwd,conv4_dgrad,conv5_fwd,conv5_dgrad,fc6_fwd,fc7_fwd,fc6_dgrad,vgg.c1_2_fwd,vgg.c1_2_dgrad,vgg.c2_2_fwd,vgg.c2_2_dgrad,vgg.c3_2_fwd,vgg.c3_2_dgrad,vgg.c4_2_fwd,vgg.c4_2_dgrad,vgg.c5_fwd,vgg.c5_dgrad \
  > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r4f/probe.jsonl"):
    d = json.loads(l); us = {k[:-3]: v for k, v in d.items() if k.endswith("_us")}
    best = min(us, key=us.get)
    print(d["op"], " ".join(f"{k}={v}" for k, v in us.items()), "best", best)
PY
bash tools/pmc_tiles.sh r4sq sq8192_fwd 21 110 113 && cat gpurun_out/pmct_r4sq/summary.txt
bash tools/pmc_tiles.sh r4c42 vgg_c4_2_fwd 110 113 114 && cat gpurun_out/pmct_r4c42/summary.txt
bash tools/pmc_tiles.sh r4c3 conv3_fwd 113 114 && cat gpurun_out/pmct_r4c3/summary.txt
