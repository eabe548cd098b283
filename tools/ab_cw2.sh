# A/B: tile choice of the LDS-DMA conv weight-grad for conv4/conv5 (others on the register kernel, REG = 99)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/t17; mkdir -p $O
python - <<'PY'
import json
K = {"c2": "cw|256|27|27|96|256|5|5|1|2|2|2", "c3": "cw|256|13|13|256|384|3|3|1|1|1|1",
     "c4": "cw|256|13|13|384|384|3|3|1|1|1|2", "c5": "cw|256|13|13|384|256|3|3|1|1|1|2"}
cfg = {"c4t1": {"c4": 1}, "c4t17": {"c4": 17}, "c4t13": {"c4": 13}, "c4t2": {"c4": 2},
       "c4t1c5t1": {"c4": 1, "c5": 1}, "c4t1c5t17": {"c4": 1, "c5": 17}, "c4t1c3t17": {"c4": 1, "c3": 17}}
for name, sel in cfg.items():
    json.dump({k: sel.get(n, 99) for n, k in K.items()}, open(f"gpurun_out/t17/{name}.json", "w"))
PY
B=cf,cr,cd,fc,fw
C="base:$B"
for n in c4t1 c4t17 c4t13 c4t2 c4t1c5t1 c4t1c5t17 c4t1c3t17; do C="$C $n:$B,cw:db=$O/$n.json"; done
timeout -k 10 500 python -u benchmarks/ab_step.py --rounds 21 --configs $C > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
