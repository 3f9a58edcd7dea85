#!/bin/bash
# GPU pass: every bench config (one JSON line each) + the per-call latency sweep, logs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
run() {  # name, args...
  local name=$1; shift
  echo "== $name: $*"
  timeout -k 10 400 python3 bench.py "$@" > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | cut -c1-600
}
run uniform4k
run zipf --config zipf
run zipf_crc32 --config zipf --algo crc32
run verify4k --config verify4k
run verify4k_host --config verify4k_host --steps 5 --warmup 1
run host4k --config host4k --steps 5 --warmup 1
run host4k_pageable --config host4k --pageable --steps 5 --warmup 1
run gloo2 --gpus 2 --dist-backend gloo --no-cpu-baseline
echo "== resume latency"; timeout -k 10 300 ./tools/resume_latency > $O/call_latency.log 2>&1 || { cat $O/call_latency.log; exit 1; }
cat $O/call_latency.log
