#!/bin/bash
# Entry-size sweep of the second session's build (uniform at every lane count, plan, direct).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03v; mkdir -p $O; cd $R
echo "== size sweep"; timeout -k 10 900 python3 -u tools/size_sweep.py > $O/size_sweep.log 2>&1 || { tail -5 $O/size_sweep.log; exit 1; }
tail -5 $O/size_sweep.log
echo done
