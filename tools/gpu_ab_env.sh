#!/bin/bash
# bench.py of one model under several env settings (same box): bash tools/gpu_ab_env.sh model batch "ENV=.. ENV2=.." ...
set -o pipefail
M=$1; B=$2; shift 2
mkdir -p gpurun_out/abenv
for e in "$@"; do
  r=$(env $e timeout -k 10 200 python bench.py --model $M --batch $B --steps 30 --warmup 8 $BENCH_ARGS 2>>gpurun_out/abenv/err | tail -1) || { tail gpurun_out/abenv/err; exit 1; }
  echo "{\"env\": \"$e\", \"model\": \"$M\", \"ms\": $(echo $r | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')}"
done
