#!/bin/bash
# GPU pass: the tests named in $1 (pytest -k), then a rocprofv3 kernel-stats run of the verify4k bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${1:-stream_release}" > $O/pt_sel.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pt_sel.log | tail -20; tail -3 $O/pt_sel.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profv -o verify -- python3 $R/bench.py --config verify4k --no-cpu-baseline --steps 20 --warmup 5 > $O/rocprofv.log 2>&1 || exit 1
tail -1 $O/rocprofv.log | cut -c1-300
find $O/profv -name '*kernel_stats.csv' -exec cat {} \;
