#!/bin/bash
# Stream scratch on hipMalloc instead of the stream-ordered pool: GPU suite, A/B against HEAD's build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03m; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_lt1k indexed4k uniform4k verify4k package4k"
L3=tools/variants/lib_pkgpass.so
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_head.so $L3 > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
grep median $O/ab1.log
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py $L3 tools/variants/lib_head.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
grep median $O/ab2.log
echo "== host big"; SIZES="128 256" REPS=4 timeout -k 10 300 python3 tools/diag_host_big.py > $O/host_big.log 2>&1; rc=$?; grep -v amdgpu.ids $O/host_big.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo ok
