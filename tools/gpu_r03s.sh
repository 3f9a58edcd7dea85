#!/bin/bash
# Long chunks with unconditional loads only (chunk_fold<LONG>): plan parity tests, then a
# same-process A/B against the previous commit and the tail-uncond-only build, two library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03s; mkdir -p $O; cd $R
echo "== pytest plan/zipf/golden"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_entrylog.py -k "plan or zipf or golden or verify or ragged or entrylog or indexed" > $O/pytest_plan.log 2>&1; rc=$?
tail -3 $O/pytest_plan.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_crc32 zipf_lt1k zipf_heads zipf_heads_sorted heads_aligned chunk4s mixed1k indexed4k uniform4k"
echo "== ab order 1"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_prev.so tools/variants/lib_tailu.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_tailu.so tools/variants/lib_prev.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo done
