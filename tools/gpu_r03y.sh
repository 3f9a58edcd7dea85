#!/bin/bash
# Second-box numbers for the round's tree: the driver's command, 100/50, Zipf CRC32C / CRC32.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03y; mkdir -p $O; cd $R
echo "== driver cmd"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
echo "== bench 100/50"; timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_100.log 2>&1 || { tail -5 $O/bench_100.log; exit 1; }
tail -1 $O/bench_100.log | cut -c1-200
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf --no-cpu-baseline --no-buckets > $O/bench_zipf.log 2>&1 || { tail -5 $O/bench_zipf.log; exit 1; }
tail -1 $O/bench_zipf.log | cut -c1-200
echo "== zipf crc32"; timeout -k 10 300 python3 bench.py --config zipf --algo crc32 --no-cpu-baseline --no-buckets > $O/bench_zipf_crc32.log 2>&1 || { tail -5 $O/bench_zipf_crc32.log; exit 1; }
tail -1 $O/bench_zipf_crc32.log | cut -c1-200
echo done
