#!/bin/bash
# Long host entries on the GPU route after the fix: suite, repeated-call diagnostic, per-call latency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03l; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== host big"; SIZES="64 128 256 512" REPS=6 timeout -k 10 300 python3 tools/diag_host_big.py > $O/host_big_fixed.log 2>&1; rc=$?; grep -v amdgpu.ids $O/host_big_fixed.log; [ $rc -eq 0 ] || exit $rc
echo "== resume latency"; timeout -k 10 300 ./tools/resume_latency > $O/call_latency.log 2>&1; rc=$?; cat $O/call_latency.log; [ $rc -eq 0 ] || exit $rc
