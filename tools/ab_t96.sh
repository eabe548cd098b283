# 96-row LDS-DMA tiles for conv1 forward: kernel timing + error vs the register kernel, then whole-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/t18; mkdir -p $O
timeout -k 10 300 python -u benchmarks/gemm_glds_bench.py --ops conv1_fwd,fc6_fwd,fc8_fwd --tiles 10,9,26,27 > $O/kern.jsonl 2>$O/kern.err || { tail -20 $O/kern.err; exit 1; }
cat $O/kern.jsonl
for t in 9 26 27; do echo "{\"cr|256|227|227|4|96|11|11|4\": $t}" > $O/cr$t.json; done
B=cf,cr,cd,cw,fc,fw
timeout -k 10 300 python -u benchmarks/ab_step.py --rounds 15 --configs "base:$B" "cr9:$B:db=$O/cr9.json" "cr26:$B:db=$O/cr26.json" "cr27:$B:db=$O/cr27.json" > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
