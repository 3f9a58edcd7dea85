#!/bin/bash
# bkd_set_fold_schedule: the new parity test for both schedules, then the whole -m gpu suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03af; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "fold_schedules|passed|failed" $O/pytest_gpu.log | tail -3; exit $rc
