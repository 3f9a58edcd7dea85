#!/bin/bash
# FETCH_SIZE per dispatch of the CRC kernels for several bench configs (args: bench arg strings)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcfetch; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
k=0
for a in "$@"; do
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c$k -o p -- python3 $R/bench.py $a --steps 3 --warmup 1 --no-cpu-baseline > $O/c$k.log 2>&1 || { echo "fail $a"; tail -5 $O/c$k.log; exit 1; }
  python3 - "$a" $O/c$k <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(list)
for p in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        v[(r["Kernel_Name"].split("(")[0].replace("void ", "")[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
print(sys.argv[1])
for (kn, c), x in sorted(v.items()):
    x = sorted(x); print("   %-42s %-11s %14.0f KB" % (kn, c, x[len(x)//2]))
PY
  k=$((k+1))
done
