#!/bin/bash
# Short-tail prefetch depth and the three-set uniform short loop: the -m gpu suite on the default
# build, then a same-process A/B of the default (short tail of <= 4-step chunks, three sets), the
# round-3 head build, kShortPF 2 / 5 and the single-prefetch chunk schedule, in two library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03r; mkdir -p $O; cd $R
echo "== pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_crc32 zipf_lt1k zipf_heads zipf_heads_sorted chunk1s chunk2s chunk4s mixed1k indexed4k uniform4k u32_l1 u64_l4 u128_l4 u128_l8 u256_l4 u256_l8 u512_l8"
V="tools/variants/lib_head.so tools/variants/lib_noshort.so tools/variants/lib_spf2.so tools/variants/lib_spf5.so"
echo "== ab order 1"
AB_ROUNDS=4 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so $V > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=4 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_spf5.so tools/variants/lib_spf2.so tools/variants/lib_noshort.so tools/variants/lib_head.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo done
