#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_zipf -o z -- python3 $R/bench.py --config zipf --steps 10 ${ZARGS} > $O/prof_zipf.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_zipf/z_kernel_stats.csv')):
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(4), '%10.1f us' % (float(r['AverageNs'])/1e3))
"
