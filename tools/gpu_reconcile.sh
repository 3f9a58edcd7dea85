#!/bin/bash
# the driver's exact command three times, the builder's 100/50 command three
# times, per-launch ramp diagnostics, and a rocprofv3 kernel trace of the driver's command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/reconcile; mkdir -p $O; cd $R
for k in 1 2 3; do
  echo "== driver cmd run $k"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$k.log 2>&1 || { tail -5 $O/driver_$k.log; exit 1; }
  tail -1 $O/driver_$k.log | cut -c1-300
done
for k in 1 2 3; do
  echo "== builder cmd run $k"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 100 --warmup 50 --no-cpu-baseline > $O/builder_$k.log 2>&1 || { tail -5 $O/builder_$k.log; exit 1; }
  tail -1 $O/builder_$k.log | cut -c1-300
done
echo "== ramp"; timeout -k 10 120 python3 tools/ramp.py > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
cut -c1-600 $O/ramp.log
echo "== ramp touch"; timeout -k 10 120 python3 tools/ramp.py --touch > $O/ramp_touch.log 2>&1 || { tail -5 $O/ramp_touch.log; exit 1; }
cut -c1-600 $O/ramp_touch.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof driver cmd"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o bench -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocprof_driver.log 2>&1 || { tail -5 $O/rocprof_driver.log; exit 1; }
tail -1 $O/rocprof_driver.log | cut -c1-300
echo done
