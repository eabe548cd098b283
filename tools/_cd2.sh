set -o pipefail
mkdir -p gpurun_out/dp1
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 120 --timeout-method thread -k "fullc" > gpurun_out/dp1/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|err " gpurun_out/dp1/tests.log | tail -20; exit $rc
