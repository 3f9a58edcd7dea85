#!/bin/bash
# Long host buffers over the host pool: GPU suite, then per-call resume latency by route up to 256 MiB.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03j; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== resume latency"; timeout -k 10 300 ./tools/resume_latency > $O/call_latency.log 2>&1 || { cat $O/call_latency.log; exit 1; }
cat $O/call_latency.log
