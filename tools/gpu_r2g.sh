#!/bin/bash
set -o pipefail
OUT=gpurun_out/r2g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_layer_kernels_gpu.py tests/test_models.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model inception_v1 --batch 128 --steps 20 --warmup 5 > $OUT/bench_incep.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench_incep.json
bash tools/gpu_prof_model.sh incep2 inception_v1 128 > /dev/null
python3 - <<'PY'
rows=[l for l in open('gpurun_out/prof_incep2/kernels.md') if l.startswith('| `')]
agg={}
for l in rows:
    parts=[p.strip() for p in l.split('|')]
    name=parts[1].strip('`').split('<')[0]
    agg[name]=agg.get(name,0)+float(parts[4])
for k,v in sorted(agg.items(), key=lambda t:-t[1])[:14]:
    print(f"{k:30s} {v/13*1000:8.1f} us/step")
PY
head -1 gpurun_out/prof_incep2/kernels.md
