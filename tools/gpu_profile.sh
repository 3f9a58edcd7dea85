#!/bin/bash
# GPU pass: parity tests -> bench -> rocprofv3 kernel-trace stats -> PMC passes (FETCH, WRITE).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r1}
mkdir -p $O
cd $R
echo "== pytest gpu"; timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf --steps 10 > $O/bench_zipf.log 2>&1 || exit 1; tail -1 $O/bench_zipf.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $O/rocprof_$TAG.log 2>&1 || exit 1
echo "== pmc fetch"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$TAG -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_fetch_$TAG.log 2>&1 || exit 1
echo "== pmc write"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$TAG -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/pmc_write_$TAG.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py $O/pmc_fetch_$TAG $O/pmc_write_$TAG uniform4k $((1048576*4100))
