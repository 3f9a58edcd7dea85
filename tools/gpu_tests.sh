#!/bin/bash
# GPU pass: the -m gpu suite (or the files/args given) with per-test timeouts, then smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu $*"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${@:-tests} > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest_gpu.log | tail -40; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
