#!/bin/bash
# GPU pass: parity tests -> bench (uniform, zipf) -> rocprofv3 kernel-trace stats -> PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate runs, kernel-trace only) for uniform4k and zipf.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${1:-r1}
mkdir -p $O
cd $R
echo "== pytest gpu"; timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf > $O/bench_zipf.log 2>&1 || exit 1; tail -1 $O/bench_zipf.log
cd /tmp && export TMPDIR=/tmp
echo "== rocprof stats"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o bench -- python3 $R/bench.py --no-cpu-baseline > $O/rocprof_$TAG.log 2>&1 || exit 1
echo "== rocprof stats zipf"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profz_$TAG -o zipf -- python3 $R/bench.py --config zipf --no-buckets > $O/rocprofz_$TAG.log 2>&1 || exit 1
for cfg in uniform4k zipf; do
  extra="--no-cpu-baseline"; [ $cfg = zipf ] && extra="--config zipf --no-buckets"
  echo "== pmc fetch $cfg"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_${cfg}_$TAG -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1 > $O/pmc_fetch_${cfg}_$TAG.log 2>&1 || exit 1
  echo "== pmc write $cfg"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_${cfg}_$TAG -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1 > $O/pmc_write_${cfg}_$TAG.log 2>&1 || exit 1
done
cd $R
python3 tools/pmc_summary.py $O/pmc_fetch_uniform4k_$TAG $O/pmc_write_uniform4k_$TAG uniform4k $((1048576*4100)) || exit 1
ZB=$(python3 -c "from bench import zipf_index; o,l=zipf_index(1<<20); print(int(o[-1]+l[-1]) + 16*len(o))")
python3 tools/pmc_summary.py $O/pmc_fetch_zipf_$TAG $O/pmc_write_zipf_$TAG zipf $ZB bkd::crc_plan_chunks_kernel || exit 1
cp profiles/pmc_uniform4k.json profiles/pmc_zipf.json $O/
