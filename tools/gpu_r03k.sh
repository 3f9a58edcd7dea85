#!/bin/bash
# A 256 MiB per-call resume differed between routes (r03j): find the route.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03k; mkdir -p $O; cd $R
echo "== big entry"; timeout -k 10 300 python3 tools/diag_big_entry.py > $O/big.log 2>&1; rc=$?; cat $O/big.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
echo "== resume latency"; timeout -k 10 300 ./tools/resume_latency > $O/call_latency.log 2>&1; cat $O/call_latency.log | tail -4
