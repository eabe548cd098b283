#!/bin/bash
# GoogLeNet (Inception-v1) and VGG-16 1-GPU training throughput + GoogLeNet kernel profile.
#   bash tools/gpu_models.sh <tag>
set -o pipefail
TAG=${1:-models}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model inception_v1 --batch 128 --steps 20 --warmup 5 > $OUT/bench_inception.json 2> $OUT/bench_inception.err || { echo "inception bench failed"; tail -20 $OUT/bench_inception.err; exit 1; }
cat $OUT/bench_inception.json
timeout -k 10 300 python -u bench.py --model vgg16 --batch 64 --steps 20 --warmup 5 > $OUT/bench_vgg16.json 2> $OUT/bench_vgg16.err || { echo "vgg bench failed"; tail -20 $OUT/bench_vgg16.err; exit 1; }
cat $OUT/bench_vgg16.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --model inception_v1 --batch 128 --steps 8 --warmup 4 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 12 --md $OUT/kernels_inception.md > /dev/null && head -3 $OUT/kernels_inception.md
