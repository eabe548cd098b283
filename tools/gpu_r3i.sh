#!/bin/bash
set -o pipefail
bash tools/pmc_ops.sh c2 conv1c3_wgrad > /dev/null 2>&1
cd gpurun_out/pmcops_c2 && for p in 1 2 3 4; do python3 - <<PY
import csv,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open('conv1c3_wgrad_p$p/p_counter_collection.csv')):
    if 'rowrun' in r['Kernel_Name']:
        d[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in d.items(): print(k, sum(v)/len(v) if v else 0, len(v))
PY
done
