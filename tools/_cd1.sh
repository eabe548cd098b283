set -o pipefail
for i in 1 2; do
timeout -k 10 120 python bench.py --steps 30 --warmup 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b256', d['ms_per_step'], d['value'])" || exit 1
done
timeout -k 10 120 python bench.py --steps 30 --warmup 10 --batch 32 --scaling strong 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b32', d['ms_per_step'], d['value'])" || exit 1
OUT=gpurun_out/r6prof2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof --steps 30 --md $OUT/kernels.md > /dev/null && head -30 $OUT/kernels.md
rm -rf $OUT/prof
