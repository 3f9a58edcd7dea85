#!/bin/bash
# Round-3 (second session) measurement pass on the committed tree: smoke, bench lines (driver's
# command twice, 100/50, Zipf CRC32C / CRC32, verify/package), rocprofv3 kernel stats for the
# headline and Zipf, PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) for both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03u; mkdir -p $O; cd $R
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }; tail -1 $O/smoke.log
for k in 1 2; do
  echo "== driver cmd $k"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$k.log 2>&1 || { tail -5 $O/bench_driver_$k.log; exit 1; }
  tail -1 $O/bench_driver_$k.log | cut -c1-200
done
echo "== bench 100/50"; timeout -k 10 200 python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_100.log 2>&1 || { tail -5 $O/bench_100.log; exit 1; }
tail -1 $O/bench_100.log | cut -c1-200
echo "== zipf"; timeout -k 10 300 python3 bench.py --config zipf > $O/bench_zipf.log 2>&1 || { tail -5 $O/bench_zipf.log; exit 1; }
tail -1 $O/bench_zipf.log | cut -c1-200
echo "== zipf crc32"; timeout -k 10 300 python3 bench.py --config zipf --algo crc32 > $O/bench_zipf_crc32.log 2>&1 || { tail -5 $O/bench_zipf_crc32.log; exit 1; }
tail -1 $O/bench_zipf_crc32.log | cut -c1-200
echo "== verify4k"; timeout -k 10 300 python3 bench.py --config verify4k > $O/bench_verify4k.log 2>&1 || { tail -5 $O/bench_verify4k.log; exit 1; }
tail -1 $O/bench_verify4k.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
echo "== rocprof stats driver cmd"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_u -o uniform4k -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/rocprof_u.log 2>&1 || exit 1
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
echo "== done"
