set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/t15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u benchmarks/tune_db.py --models alexnet:256 --out $O/tune_reg.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/t15/tune_reg.json"))
print("REG picks:", {k: v for k, v in d.items() if v == 99})
json.dump({k: v for k, v in d.items() if v != 99}, open("gpurun_out/t15/tune_noreg.json", "w"))
PY
timeout -k 10 500 python -u benchmarks/ab_step.py --rounds 7 --configs "base:cf,cr,cd,fc,fw" "reg:cf,cr,cd,fc,fw:db=$O/tune_reg.json" "noreg:cf,cr,cd,fc,fw:db=$O/tune_noreg.json" > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
