#!/bin/bash
# First GPU pass: smoke -> gpu parity tests -> bench -> lane sweep -> rocprofv3 kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; cat $O/smoke.log | tail -5; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1; rc=$?; tail -3 $O/bench.log; [ $rc -eq 0 ] || exit $rc
for L in 4 8 16 32; do echo "== lanes $L"; timeout -k 10 200 python3 bench.py --no-cpu-baseline --lanes $L --steps 20 > $O/bench_l$L.log 2>&1 || exit 1; tail -1 $O/bench_l$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['achieved'], d['roofline']['avg_kernel_ms'])"; done
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf --steps 10 > $O/bench_zipf.log 2>&1; tail -1 $O/bench_zipf.log
echo "== rocprof"; cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $O/rocprof.log 2>&1; rc=$?; tail -3 $O/rocprof.log; find $O/prof -name "*stats*" | head; exit $rc
