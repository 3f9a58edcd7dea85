#!/bin/bash
# Round-3 measurement pass: GPU suite, A/B of the long-entry tail-load gate against lib_r02,
# bench lines (headline in the driver's form, Zipf CRC32C / CRC32 with cpu_baseline), rocprofv3
# kernel stats and PMC traffic (FETCH_SIZE / WRITE_SIZE in separate passes) for uniform4k and zipf.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03h; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="uniform4k u512_l8 u1024_l8 u2048_l8 u8192_l8 u16384_l16 indexed4k zipf"
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_r02.so > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
grep median $O/ab1.log
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 400 python3 tools/ab_libs.py tools/variants/lib_r02.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
grep median $O/ab2.log
echo "== driver cmd"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-300
echo "== bench 100/50"; timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 > $O/bench_100.log 2>&1 || { tail -5 $O/bench_100.log; exit 1; }
tail -1 $O/bench_100.log | cut -c1-300
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf > $O/bench_zipf.log 2>&1 || { tail -5 $O/bench_zipf.log; exit 1; }
tail -1 $O/bench_zipf.log | cut -c1-300
echo "== zipf crc32"; timeout -k 10 300 python3 bench.py --config zipf --algo crc32 > $O/bench_zipf_crc32.log 2>&1 || { tail -5 $O/bench_zipf_crc32.log; exit 1; }
tail -1 $O/bench_zipf_crc32.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
echo "== rocprof stats uniform4k"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_u -o uniform4k -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/rocprof_u.log 2>&1 || exit 1
echo "== rocprof stats zipf"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_z -o zipf -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline > $O/rocprof_z.log 2>&1 || exit 1
for cfg in uniform4k zipf; do
  extra="--no-cpu-baseline"; [ $cfg = zipf ] && extra="--config zipf --no-buckets --no-cpu-baseline"
  echo "== pmc fetch $cfg"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$cfg -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1 > $O/pmc_fetch_$cfg.log 2>&1 || exit 1
  echo "== pmc write $cfg"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$cfg -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1 > $O/pmc_write_$cfg.log 2>&1 || exit 1
done
cd $R
python3 tools/pmc_summary.py $O/pmc_fetch_uniform4k $O/pmc_write_uniform4k uniform4k $((1048576*4100)) > $O/pmc_u.json || exit 1
ZB=$(python3 -c "from bench import zipf_index; o,l=zipf_index(1<<20); print(int(o[-1]+l[-1]) + 16*len(o))")
python3 tools/pmc_summary.py $O/pmc_fetch_zipf $O/pmc_write_zipf zipf $ZB bkd::crc_plan_chunks_kernel > $O/pmc_z.json || exit 1
cp profiles/pmc_uniform4k.json profiles/pmc_zipf.json $O/
echo "== done"
