set -o pipefail
mkdir -p gpurun_out/cd8
timeout -k 10 300 python -u -m pytest tests/test_conv_direct_gpu.py tests/test_tune_table_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cd8/tests.log 2>&1; rc=$?; tail -3 gpurun_out/cd8/tests.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python bench.py --steps 30 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('direct', d['ms_per_step'], d['value'])" || exit 1
CXXNET_CONV_DIRECT=0 timeout -k 10 120 python bench.py --steps 30 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gemm', d['ms_per_step'], d['value'])" || exit 1
done
