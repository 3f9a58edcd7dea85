#!/bin/bash
# Short-tail v2 (three register sets, wave-uniform exit): plan parity tests, then a same-process
# A/B against the single-prefetch schedule (tools/variants/lib_noshort.so) in both library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03q; mkdir -p $O; cd $R
echo "== pytest plan/zipf/golden"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "plan or zipf or golden or verify or ragged" > $O/pytest_plan.log 2>&1; rc=$?
tail -3 $O/pytest_plan.log; [ $rc -eq 0 ] || exit $rc
echo "== ab order 1"
AB_ROUNDS=4 AB_WORK="zipf zipf_crc32 zipf_lt1k zipf_heads zipf_heads_sorted heads_aligned heads_sep chunk1s chunk2s chunk4s mixed1k indexed4k uniform4k" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_noshort.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log | grep -v "^u"
echo "== ab order 2"
AB_ROUNDS=4 AB_WORK="zipf zipf_crc32 zipf_lt1k zipf_heads zipf_heads_sorted heads_aligned heads_sep chunk1s chunk2s chunk4s mixed1k indexed4k uniform4k" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_noshort.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log | grep -v "^u"
echo done
