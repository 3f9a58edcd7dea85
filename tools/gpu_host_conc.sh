#!/bin/bash
# GPU pass: host-staging tests, then concurrent host-verify callers with 1 and 4 staging sets.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "host or concurrent" > $O/pt_host.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pt_host.log | tail -30; tail -2 $O/pt_host.log; [ $rc -eq 0 ] || exit $rc
for B in 64 1024; do
  BKD_HOST_STAGES=1 timeout -k 10 300 python3 tools/host_concurrency.py $B 2>&1 | tee -a $O/host_conc.log || exit 1
  timeout -k 10 300 python3 tools/host_concurrency.py $B 2>&1 | tee -a $O/host_conc.log || exit 1
done
