#!/bin/bash
# Final tree: -m gpu suite, smoke, the driver's command twice, 100/50, rocprofv3 kernel stats of the
# driver's command, launch ramp with the clock probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ae; mkdir -p $O; cd $R
echo "== pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }; tail -1 $O/smoke.log
for k in 1 2; do
  echo "== driver cmd $k"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$k.log 2>&1 || { tail -5 $O/bench_driver_$k.log; exit 1; }
  tail -1 $O/bench_driver_$k.log | cut -c1-200
done
echo "== bench 100/50"; timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_100.log 2>&1 || { tail -5 $O/bench_100.log; exit 1; }
tail -1 $O/bench_100.log | cut -c1-200
echo "== ramp"; timeout -k 10 300 python3 tools/ramp_clock.py --probe --rounds 2 > $O/ramp_clock.log 2>&1 || { tail -5 $O/ramp_clock.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
echo "== rocprof stats driver cmd"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_u -o uniform4k -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/rocprof_u.log 2>&1 || exit 1
echo done
