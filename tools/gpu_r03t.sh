#!/bin/bash
# Indexed short-entry class with three register sets and countable waits: the -m gpu suite, then a
# same-process A/B (new / previous commit, each also with the class forced on for every batch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03t; mkdir -p $O; cd $R
echo "== pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="packed64 packed64_64m chunk1s chunk2s zipf zipf_crc32 zipf_lt1k mixed1k uniform1k_idx indexed4k"
V="tools/variants/lib_prev.so tools/variants/lib_newforce.so tools/variants/lib_prevforce.so"
echo "== ab order 1"
AB_ROUNDS=4 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so $V > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=4 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_prevforce.so tools/variants/lib_newforce.so tools/variants/lib_prev.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo done
