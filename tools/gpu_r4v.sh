#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 60 python -u tools/diag_memset_graph.py 2>&1 | grep -v amdgpu
echo "== graph vs eager"; DIAG_EAGER=1 timeout -k 10 200 python -u tools/diag_e2e.py 2>&1 | grep -v amdgpu | cut -c1-200 | head -12
bash tools/gpu_r4u.sh
