#!/bin/bash
# Chunk-kernel variants A/B in one process (both library orders): unconditional tail loads,
# 4 halves per loop iteration, early prefetch, and both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03f; mkdir -p $O; cd $R
W="zipf zipf_heads_sorted chunk1s chunk4s mixed1k indexed4k uniform4k verify4k package4k"
V="tools/variants/lib_tailu.so tools/variants/lib_unroll4.so tools/variants/lib_early.so tools/variants/lib_tailu_unroll4.so"
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 500 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so $V > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
grep median $O/ab1.log
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 500 python3 tools/ab_libs.py $(echo $V | tr ' ' '\n' | tac | tr '\n' ' ') bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
grep median $O/ab2.log
