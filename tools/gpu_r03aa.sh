#!/bin/bash
# Config 4's per-GPU shard at N = 1 (the per-GPU workload of the driver's N > 1 runs), the driver's
# step counts, and 100/50.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03aa; mkdir -p $O; cd $R
echo "== shard8m 20/5"; timeout -k 10 300 python3 bench.py --config shard8m --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_shard8m.log 2>&1 || { tail -5 $O/bench_shard8m.log; exit 1; }
tail -1 $O/bench_shard8m.log | cut -c1-300
echo "== shard8m 100/20"; timeout -k 10 300 python3 bench.py --config shard8m --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_shard8m_100.log 2>&1 || { tail -5 $O/bench_shard8m_100.log; exit 1; }
tail -1 $O/bench_shard8m_100.log | cut -c1-300
echo done
