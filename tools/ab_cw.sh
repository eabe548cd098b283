# A/B: LDS-DMA conv weight-grad per layer vs the register-staged kernel (REG = 99) on AlexNet b256
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/t16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "conv or wgrad" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
python - <<'PY'
import json
K = {"c2": "cw|256|27|27|96|256|5|5|1|2|2|2", "c3": "cw|256|13|13|256|384|3|3|1|1|1|1",
     "c4": "cw|256|13|13|384|384|3|3|1|1|1|2", "c5": "cw|256|13|13|384|256|3|3|1|1|1|2"}
def tab(glds):  # layers in `glds` on LDS-DMA tile 1, the rest on the register kernel
    return {k: (1 if n in glds else 99) for n, k in K.items()}
for name, g in {"reg": [], "c4": ["c4"], "c24": ["c2", "c4"], "c234": ["c2", "c3", "c4"], "all": list(K)}.items():
    json.dump(tab(g), open(f"gpurun_out/t16/cw_{name}.json", "w"))
PY
B=cf,cr,cd,fc,fw
timeout -k 10 500 python -u benchmarks/ab_step.py --rounds 7 --configs "base:$B" "reg:$B,cw:db=$O/cw_reg.json" "c4:$B,cw:db=$O/cw_c4.json" "c24:$B,cw:db=$O/cw_c24.json" "c234:$B,cw:db=$O/cw_c234.json" "all:$B,cw:db=$O/cw_all.json" > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
