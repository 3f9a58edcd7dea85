#!/bin/bash
# Round 3, second pass: GPU suite, thread scaling A/B (r02 lib vs now), per-J head costs, host-route
# bench lines, and kernel stats + PMC traffic for the verify and package routes on their own.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03b; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== thread scaling"; timeout -k 10 300 ./tools/thread_scaling tools/variants/lib_r02.so bookkeeper_amd/libbkdigest.so tools/variants/lib_r02.so bookkeeper_amd/libbkdigest.so > $O/thread_scaling.log 2>&1 || { tail -5 $O/thread_scaling.log; exit 1; }
cat $O/thread_scaling.log
echo "== heads by J"; timeout -k 10 300 python3 tools/diag_heads_j.py > $O/heads_j.log 2>&1 || { tail -5 $O/heads_j.log; exit 1; }
cat $O/heads_j.log
for cfg in "verify4k_host" "verify4k_host --algo crc32" "host4k" "host4k --pageable"; do
  tag=$(echo $cfg | tr ' -' '__')
  echo "== bench $cfg"; timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 2 > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | cut -c1-900
done
cd /tmp && export TMPDIR=/tmp
for op in verify package; do
  echo "== rocprof stats $op"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$op -o $op -- python3 $R/bench.py --config verify4k --digest-op $op --steps 20 --warmup 5 > $O/rocprof_$op.log 2>&1 || { tail -5 $O/rocprof_$op.log; exit 1; }
  tail -1 $O/rocprof_$op.log | cut -c1-400
  echo "== pmc fetch $op"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$op -o pmc -- python3 $R/bench.py --config verify4k --digest-op $op --steps 5 --warmup 1 > $O/pmc_fetch_$op.log 2>&1 || { tail -5 $O/pmc_fetch_$op.log; exit 1; }
  echo "== pmc write $op"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$op -o pmc -- python3 $R/bench.py --config verify4k --digest-op $op --steps 5 --warmup 1 > $O/pmc_write_$op.log 2>&1 || { tail -5 $O/pmc_write_$op.log; exit 1; }
done
cd $R
echo "== ramp A/B (xor3 main fold vs plain)"
for lib in bookkeeper_amd/libbkdigest.so tools/variants/lib_xor3.so bookkeeper_amd/libbkdigest.so tools/variants/lib_xor3.so; do
  timeout -k 10 120 python3 tools/ramp.py --lib $lib --rounds 2 --idle-ms 1500 --launches 100 >> $O/ramp_ab.log 2>&1 || { tail -5 $O/ramp_ab.log; exit 1; }
done
python3 - <<'PY'
import json, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/r03b"
for line in open(os.path.join(O, "ramp_ab.log")):
    if line.startswith("{"):
        d = json.loads(line)
        print(d["lib"], d["round"], d["mean_0_5"], d["mean_5_25_driver_window"], d["mean_25_50"], d["mean_50_150_builder_window"])
PY
echo "== ab_libs"; AB_ROUNDS=3 timeout -k 10 600 python3 tools/ab_libs.py > $O/ab_libs.log 2>&1 || { tail -5 $O/ab_libs.log; exit 1; }
tail -30 $O/ab_libs.log
echo done
