#!/bin/bash
# Data-parallel AlexNet b256 at world 1 (RCCL forced) under reduction / gather variants, two
# interleaved passes: bash tools/gpu_dp_variants.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-dpvar}
mkdir -p $OUT
export TMPDIR=/tmp CXXNET_DIST_FORCE=1
run() {  # label, bench args...
  local lab=$1; shift
  r=$(timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29741 bench.py --steps 40 --warmup 10 "$@" 2>>$OUT/err | tail -1) || { tail -5 $OUT/err; exit 1; }
  echo "{\"variant\": \"$lab\", \"ms\": $(echo $r | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')}" | tee -a $OUT/dp.jsonl
}
for pass in 1 2; do
  run auto
  run gather0 --set fullc_gather=0
  run gather1 --set fullc_gather=1
  run shard --dp-mode shard
  run bucket256 --bucket-mb 256
done
