set -o pipefail
mkdir -p gpurun_out/dp2
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -v --timeout 200 --timeout-method thread -k "two_ranks" > gpurun_out/dp2/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|dp 2-rank" gpurun_out/dp2/tests.log | tail -30; exit 0
