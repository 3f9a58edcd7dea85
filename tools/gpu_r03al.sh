#!/bin/bash
# Heads at 4 lanes per chunk: the plan geometry 4 lanes x 64 steps (same 4 KiB chunks) against the
# default 8 x 32, on the Zipf batch, its heads alone and the sorted heads (same library, one
# process per geometry, twice in alternating order).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/${OUT:-r03al}; mkdir -p $O; cd $R
W="zipf zipf_heads zipf_heads_sorted"
for k in 1 2; do
  for g in ${GEOMS:-8,32,16 4,64,16}; do
    AB_GEOM=$g AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 300 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so > $O/geom_${g}_$k.log 2>&1 || { tail -20 $O/geom_${g}_$k.log; exit 1; }
    echo "geom $g run $k"; grep median $O/geom_${g}_$k.log
  done
done
echo done
