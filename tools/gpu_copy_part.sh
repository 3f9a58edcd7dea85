#!/bin/bash
# Host-resident verify latency / throughput against the copy-pool part size (BKD_COPY_PART_KIB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for P in 4096 1024 256 128; do
  for B in 64 256 1024; do
    echo "part ${P} KiB" >> $O/copy_part.log
    BKD_COPY_PART_KIB=$P timeout -k 10 200 python3 tools/host_concurrency.py $B >> $O/copy_part.log 2>&1 || exit 1
  done
  BKD_COPY_PART_KIB=$P timeout -k 10 300 python3 bench.py --config verify4k_host --steps 3 --warmup 1 > $O/vh_$P.log 2>&1 || exit 1
  echo "part ${P} KiB verify4k_host: $(tail -1 $O/vh_$P.log | cut -c1-200)" >> $O/copy_part.log
done
cat $O/copy_part.log
