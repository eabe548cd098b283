set -o pipefail
mkdir -p gpurun_out/r7
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -q -x -m gpu > gpurun_out/r7/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r7/tests.log; [ $rc -gt 1 ] && exit $rc
CXXNET_GEMM_PF=1 timeout -k 10 300 python benchmarks/gemm_ceiling.py > gpurun_out/r7/pf1.jsonl 2>&1 || exit 1
CXXNET_GEMM_PF=2 timeout -k 10 300 python benchmarks/gemm_ceiling.py > gpurun_out/r7/pf2.jsonl 2>&1 || exit 1
CXXNET_GEMM_PF=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7/bench_pf1.log 2>&1 || exit 1
CXXNET_GEMM_PF=2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r7/bench_pf2.log 2>&1 || exit 1
tail -1 gpurun_out/r7/bench_pf1.log; tail -1 gpurun_out/r7/bench_pf2.log
