#!/bin/bash
# Quick GPU pass: parity tests then benches (uniform, zipf crc32c, zipf crc32).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
echo "== pytest gpu"; timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for args in "--no-cpu-baseline" "--config zipf" "--config zipf --algo crc32" ${EXTRA_BENCH}; do
  echo "== bench $args"; timeout -k 10 300 python3 bench.py $args > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], 'GiB/s', d['roofline']['achieved'], 'GB/s', d['roofline']['avg_kernel_ms'], 'ms', d['roofline']['frac'])"
done
