#!/bin/bash
# GPU pass: the -m gpu suite, then a same-process A/B of the current library against
# tools/variants/lib_*.so in both library orders (AB_WORK selects the workloads).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
V=$(ls tools/variants/lib_*.so)
echo "== order 1"; timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so $V > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; cat $O/ab1.log | grep median
echo "== order 2"; timeout -k 10 600 python3 tools/ab_libs.py $V bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; cat $O/ab2.log | grep median
