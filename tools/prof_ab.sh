#!/bin/bash
# Per-kernel stats of each library on one A/B workload (AB_WORK, default zipf), one rocprofv3 run each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; cd $R; export TMPDIR=/tmp
W=${AB_WORK:-zipf}
for L in bookkeeper_amd/libbkdigest.so tools/variants/lib_*.so; do
  b=$(basename $L .so)
  AB_WORK=$W AB_ROUNDS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- python3 tools/ab_libs.py $L > $O/prof_$b.log 2>&1 || exit $?
  f=$(find $O/prof_$b -name '*kernel_stats.csv' | head -1)
  echo "== $b"; cut -d, -f1-4 $f | head -14
done
