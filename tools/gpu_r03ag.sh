#!/bin/bash
# Adaptive schedule in the fused verify kernel: the -m gpu suite (both schedules forced in
# test_fold_schedules_bit_exact), then the verify bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ag; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== verify4k"; timeout -k 10 300 python3 bench.py --config verify4k > $O/bench_verify4k.log 2>&1 || { tail -5 $O/bench_verify4k.log; exit 1; }
tail -1 $O/bench_verify4k.log | cut -c1-250
echo done
