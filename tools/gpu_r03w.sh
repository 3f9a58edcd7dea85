#!/bin/bash
# Uniform auto lane choice 256..511 B -> 8 lanes: uniform parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03w; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "uniform" > $O/pytest_uniform.log 2>&1; rc=$?
tail -3 $O/pytest_uniform.log; exit $rc
