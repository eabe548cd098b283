set -o pipefail
for d in 3 11 19 27; do CXN_CD_DBG=$d timeout -k 10 100 python benchmarks/conv_direct_probe.py --batch 256 --ops conv3 --paths direct --dirs fwd 2>&1 | grep op || exit 1; done
