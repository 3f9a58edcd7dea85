#!/bin/bash
# Uniform batches with unconditional tail loads: GPU suite, same-process A/B against the previous
# build (lib_r02: the round-2 kernels), headline bench in the driver's exact form.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03g; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
W="uniform4k u1024_l8 u512_l8 indexed4k verify4k package4k zipf"
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_r02.so > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
grep median $O/ab1.log
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py tools/variants/lib_r02.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
grep median $O/ab2.log
for k in 1 2; do
  echo "== driver cmd $k"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$k.log 2>&1 || { tail -5 $O/driver_$k.log; exit 1; }
  tail -1 $O/driver_$k.log | cut -c1-400
done
