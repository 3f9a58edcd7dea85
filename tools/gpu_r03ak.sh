#!/bin/bash
# Barrier-free plan_combine for entry blocks without entries of > 64 chunks (plan_count flags the
# others): plan parity tests, same-process A/B against the previous commit in two orders, and
# rocprofv3 kernel stats of the Zipf bench (plan kernel durations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ak; mkdir -p $O; cd $R
echo "== pytest plan"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_entrylog.py tests/test_gpu_streams_host.py -k "plan or zipf or golden or verify or ragged or entrylog or indexed or short or big or geometr" > $O/pytest_plan.log 2>&1; rc=$?
tail -2 $O/pytest_plan.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_crc32 zipf_heads mixed1k chunk1s packed64_64m indexed4k"
echo "== ab order 1"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_prev.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_prev.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof zipf"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_z -o zipf -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline > $O/rocprof_z.log 2>&1 || exit 1
echo done
