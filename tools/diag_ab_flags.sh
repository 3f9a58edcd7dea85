#!/bin/bash
# Same diag workloads under two BKD_PLAN_FLAGS values (A/B of a plan variant), kernel breakdown each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for F in ${FLAGS:-0 1}; do
  echo "##### BKD_PLAN_FLAGS=$F"
  export BKD_PLAN_FLAGS=$F
  bash $R/tools/diag_ragged.sh 2>&1 | grep -v "^W20\|^E20" || exit 1
done
