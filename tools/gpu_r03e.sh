#!/bin/bash
# Early prefetch of the next chunk (before waiting on the current one's blocks): GPU suite on the new
# default, then a same-process A/B against the late-prefetch build in both library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03e; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_crc32 zipf_heads zipf_heads_sorted chunk1s chunk2s chunk4s mixed1k zipf_lt1k indexed4k uniform4k verify4k package4k"
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_late.so > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
cat $O/ab1.log | grep median
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_late.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
cat $O/ab2.log | grep median
echo "== bench zipf"; timeout -k 10 300 python3 bench.py --config zipf --no-cpu-baseline > $O/bench_zipf.log 2>&1 || { tail -5 $O/bench_zipf.log; exit 1; }
tail -1 $O/bench_zipf.log | cut -c1-700
