#!/bin/bash
# One runner for every GPU-box task (run it through gpurun):  bash tools/gpu.sh <task> [args...]
#
#   check [tag]                         GPU tests, smoke(), 1-GPU bench, kernel-trace summary
#   tests [pytest args...]              the GPU test suite in one process
#   bench [bench.py args...]            bench.py with the given args (one JSON line)
#   prof <tag> [model] [batch]          rocprofv3 kernel trace of the training step -> kernels.md
#   trace <tag> [model] [batch]         per-layer GPU time (roctx range per layer) -> layers.md
#   pmc <tag> <op> <match> <cmd...>     four rocprofv3 --pmc passes over <cmd>'s kernels named
#                                       <match> -> one pmc_table.py row
#   ab-env <model> <batch> "ENV=.." ... bench.py under several environments, same box
#   ab-trees <dir> ...                  bench.py in several built worktrees (MODELS="alexnet:256 ..")
#   models [tag]                        GoogLeNet b128 + VGG-16 b64 benches and a GoogLeNet profile
#   torch-models [tag]                  eager PyTorch GoogLeNet / VGG-16 for the comparison table
#   dp [tag]                            data-parallel AlexNet b256 at world 1 (RCCL forced), variants
#   prof-dp [tag]                       kernel profiles plain vs data-parallel (world 1) + idle gaps
#   host [tag]                          host enqueue cost vs GPU time, plain and data-parallel
#   step-tune <model> <batch> [args..]  in-step tile re-tuning, then shipped vs tuned A/B
#   tune                                fill the tile table for the shipped model / batch list
#   io [tag]                            JPEG pipeline throughput: decode alone and feeding AlexNet
#
# Every GPU step runs under its own timeout; a failing step ends the call.
set -o pipefail
T=$1; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
ms() { python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])'; }

prof_bench() {  # out-dir steps-total bench args...
  local out=$1 n=$2; shift 2
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- \
     python3 $R/bench.py "$@" > $out/prof.log 2>&1) || { echo "rocprof failed"; tail -20 $out/prof.log; exit 1; }
  python3 $R/tools/prof_summary.py $out/prof --steps $n --md $out/kernels.md > /dev/null && head -40 $out/kernels.md
  rm -f $out/prof/*/run_kernel_trace.csv $out/prof/run_kernel_trace.csv 2>/dev/null
}

case $T in
check)
  OUT=gpurun_out/${1:-check}; mkdir -p $OUT
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  timeout -k 10 180 python bench.py --steps 30 --warmup 10 > $OUT/bench.json 2> $OUT/bench.err \
    || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  prof_bench $R/$OUT 18 --steps 13 --warmup 5 ;;
tests)
  mkdir -p gpurun_out/tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread "$@" \
    > gpurun_out/tests/tests.log 2>&1; rc=$?
  tail -15 gpurun_out/tests/tests.log; exit $rc ;;
bench)
  timeout -k 10 300 python bench.py "$@" ;;
prof)
  OUT=$R/gpurun_out/prof_${1:-run}; mkdir -p $OUT
  prof_bench $OUT 13 --model ${2:-alexnet} --batch ${3:-256} --steps 10 --warmup 3 ;;
trace)
  OUT=$R/gpurun_out/${1:-tr}; mkdir -p $OUT
  (cd /tmp && CXXNET_TRACE_LAYERS=1 timeout -k 10 240 rocprofv3 --marker-trace --hip-trace --kernel-trace \
     --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --model ${2:-alexnet} --batch ${3:-256} \
     --steps 5 --warmup 3 > $OUT/prof.log 2>&1) || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
  python3 tools/layer_times.py $OUT/prof --md $OUT/layers.md | head -60
  rm -f $OUT/prof/*/*hip_api_trace.csv $OUT/prof/*hip_api_trace.csv 2>/dev/null ;;
pmc)
  bash tools/pmc_cmd.sh "$@" ;;
ab-env)
  M=$1; B=$2; shift 2; mkdir -p gpurun_out/abenv
  for e in "$@"; do
    r=$(env $e timeout -k 10 200 python bench.py --model $M --batch $B --steps 30 --warmup 8 $BENCH_ARGS \
        2>>gpurun_out/abenv/err | tail -1) || { tail gpurun_out/abenv/err; exit 1; }
    echo "{\"env\": \"$e\", \"model\": \"$M\", \"ms\": $(echo $r | ms)}"
  done ;;
ab-trees)
  OUT=$R/gpurun_out/ab; mkdir -p $OUT
  for mb in ${MODELS:-alexnet:256 inception_v1:128}; do m=${mb%%:*}; b=${mb##*:}
    for d in "$@"; do
      r=$(cd $R/$d && timeout -k 10 200 python bench.py --model $m --batch $b --steps 30 --warmup 8 2>>$OUT/ab.err \
          | tail -1) || { tail $OUT/ab.err; exit 1; }
      echo "{\"tree\": \"$d\", \"model\": \"$m\", \"ms\": $(echo $r | ms)}" | tee -a $OUT/ab.jsonl
    done
  done ;;
models)
  OUT=$R/gpurun_out/${1:-models}; mkdir -p $OUT
  for mb in inception_v1:128 vgg16:64; do m=${mb%%:*}; b=${mb##*:}
    timeout -k 10 300 python -u bench.py --model $m --batch $b --steps 20 --warmup 5 > $OUT/bench_$m.json \
      2> $OUT/bench_$m.err || { echo "$m bench failed"; tail -20 $OUT/bench_$m.err; exit 1; }
    cat $OUT/bench_$m.json
  done
  prof_bench $OUT 12 --model inception_v1 --batch 128 --steps 8 --warmup 4 ;;
torch-models)
  OUT=gpurun_out/${1:-tm}; mkdir -p $OUT
  for mb in inception_v1:128 vgg16:64; do m=${mb%%:*}; b=${mb##*:}
    timeout -k 10 300 python -u benchmarks/torch_models.py --model $m --batch $b > $OUT/torch_$m.json \
      2> $OUT/torch_$m.err || { echo "torch $m failed"; tail -20 $OUT/torch_$m.err; exit 1; }
    cat $OUT/torch_$m.json
  done ;;
dp)
  OUT=gpurun_out/${1:-dpvar}; mkdir -p $OUT
  export CXXNET_DIST_FORCE=1
  run() {  # label, bench args...
    local lab=$1; shift
    r=$(timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29741 bench.py --steps 40 --warmup 10 "$@" 2>>$OUT/err | tail -1) || { tail -5 $OUT/err; exit 1; }
    echo "{\"variant\": \"$lab\", \"ms\": $(echo $r | ms)}" | tee -a $OUT/dp.jsonl
  }
  for pass in 1 2; do
    run auto; run gather0 --set fullc_gather=0; run gather1 --set fullc_gather=1; run shard --dp-mode shard
    run b32 --batch 32
  done ;;
prof-dp)
  OUT=$R/gpurun_out/${1:-profdp}; mkdir -p $OUT/plain $OUT/dp
  M=${M:-alexnet}; B=${B:-256}
  prof_bench $OUT/plain 13 --model $M --batch $B --steps 10 --warmup 3 > /dev/null
  CXXNET_DIST_FORCE=1 prof_bench $OUT/dp 13 --model $M --batch $B --steps 10 --warmup 3 > /dev/null
  head -1 $OUT/plain/kernels.md; head -1 $OUT/dp/kernels.md ;;
host)
  OUT=gpurun_out/${1:-host}; mkdir -p $OUT
  for b in 32 256; do
    for g in -1 1; do
      timeout -k 10 200 python -u benchmarks/host_overhead.py --batch $b --graph $g --steps 10 >> $OUT/host.jsonl \
        2>> $OUT/host.err || { echo "plain b$b g$g failed"; tail -5 $OUT/host.err; exit 1; }
      CXXNET_DIST_FORCE=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29731 benchmarks/host_overhead.py --batch $b --graph $g --steps 10 \
        >> $OUT/host_dp.jsonl 2>> $OUT/host.err || { echo "dp b$b g$g failed"; tail -5 $OUT/host.err; exit 1; }
    done
  done
  cat $OUT/host.jsonl $OUT/host_dp.jsonl ;;
step-tune)
  M=$1; B=$2; shift 2
  OUT=gpurun_out/st_${M}_$B; mkdir -p $OUT
  timeout -k 10 900 python -u benchmarks/step_tune.py --model $M --batch $B --steps 8 --rounds 2 \
    --out $OUT/table.json "$@" > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
  tail -3 $OUT/tune.log
  for i in 1 2 3; do
    for t in shipped tuned; do
      if [ $t = tuned ]; then export CXXNET_GEMM_TUNE_DB=$PWD/$OUT/table.json; else unset CXXNET_GEMM_TUNE_DB; fi
      r=$(timeout -k 10 200 python bench.py --model $M --batch $B --scaling strong --steps 40 --warmup 10 \
          2>>$OUT/err | tail -1) || exit 1
      echo "{\"table\": \"$t\", \"ms\": $(echo $r | ms)}" | tee -a $OUT/ab.jsonl
    done
  done ;;
tune)
  mkdir -p gpurun_out/tune
  timeout -k 10 1000 python -u benchmarks/tune_db.py --models alexnet:256,alexnet:128,alexnet:64,alexnet:32,\
inception_v1:128,inception_v1:64,vgg16:64,vgg16:32,mnist_conv:100,bowl:64 --out gpurun_out/tune/glds_tune_gfx950.json \
    > gpurun_out/tune/tune.log 2>&1 || { tail -20 gpurun_out/tune/tune.log; exit 1; }
  tail -3 gpurun_out/tune/tune.log ;;
io)
  OUT=gpurun_out/${1:-io}; mkdir -p $OUT
  D=/tmp/cxxnet_io_data
  timeout -k 10 500 python -u benchmarks/io_throughput.py --dir $D --n 4096 --workers 4,8,16 --batches 16 \
    --iters imgbin,imgbinx --modes native,process > $OUT/io_decode.jsonl 2> $OUT/io_decode.err \
    || { tail -20 $OUT/io_decode.err; exit 1; }
  cut -c1-300 $OUT/io_decode.jsonl
  timeout -k 10 400 python -u benchmarks/io_throughput.py --dir $D --workers 16 --batches 24 \
    --iters imgbin,imgbinx --modes native --train alexnet > $OUT/io_train.jsonl 2> $OUT/io_train.err \
    || { tail -20 $OUT/io_train.err; exit 1; }
  cut -c1-300 $OUT/io_train.jsonl ;;
*)
  sed -n '2,22p' $0; exit 2 ;;
esac
