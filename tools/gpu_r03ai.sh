#!/bin/bash
# Round-end rehearsal of the committed tree: -m gpu suite, smoke, the driver's command, the Zipf line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ai; mkdir -p $O; cd $R
echo "== pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }; tail -1 $O/smoke.log
echo "== driver cmd"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf > $O/bench_zipf.log 2>&1 || { tail -5 $O/bench_zipf.log; exit 1; }
tail -1 $O/bench_zipf.log | cut -c1-200
echo done
