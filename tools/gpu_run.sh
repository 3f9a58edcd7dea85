#!/bin/bash
# One parametrized GPU-box runner for the measurement and test steps (replaces the per-lease
# gpu_r03*.sh scripts). Usage, through gpurun:
#   tools/gpu_run.sh TAG STEP [STEP ...]
# Logs go to gpurun_out/TAG/; the first failing step ends the run (no GPU step after a failure).
# Steps:
#   tests            pytest -m gpu (the driver's suite)        tests:EXPR  only tests matching -k EXPR
#   smoke            __graft_entry__.smoke()
#   driver           bench.py --gpus 1 --steps 20 --warmup 5 (the driver's command)
#   trace            the driver's command with --trace-launches (HIP events around every launch)
#   bench100         bench.py --steps 100 --warmup 50
#   zipf | zipf32    bench.py --config zipf [--algo crc32]
#   verify | shard8m bench.py --config verify4k | shard8m
#   stats_uniform | stats_zipf   rocprofv3 --kernel-trace --stats of the driver's command / zipf
#   pmc_uniform | pmc_zipf       FETCH_SIZE and WRITE_SIZE passes (separate) + tools/pmc_summary.py
#   pmc_verify | pmc_package     the same for bench.py --config verify4k --digest-op verify | package
#   stats_verify | stats_package rocprofv3 --kernel-trace --stats of one framed route
#   ab:LIBS          tools/ab_libs.py over the comma-separated libs (AB_WORK selects workloads)
#   kstats:LIB       rocprofv3 kernel stats of tools/ab_libs.py on one library (AB_WORK workloads)
#   py:SCRIPT        python3 SCRIPT (a tools/ diagnostic)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
run() {  # run NAME SECONDS CMD...: one GPU step under its own time limit
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  tail -n 2 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; exit $rc; fi
}
ZB=""
zipf_bytes() { [ -n "$ZB" ] || ZB=$(python3 -c "from bench import zipf_index; o,l=zipf_index(1<<20); print(int(o[-1]+l[-1]) + 16*len(o))"); }
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    tests:*) run pytest_gpu_sel 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${step#tests:}" ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) run bench_driver 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    trace) run bench_driver_trace 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --trace-launches ;;
    bench100) run bench_100 200 python3 bench.py --steps 100 --warmup 50 --no-cpu-baseline ;;
    zipf) run bench_zipf 300 python3 bench.py --config zipf ;;
    zipf32) run bench_zipf_crc32 300 python3 bench.py --config zipf --algo crc32 ;;
    verify) run bench_verify4k 300 python3 bench.py --config verify4k ;;
    shard8m) run bench_shard8m 300 python3 bench.py --config shard8m ;;
    stats_uniform) (cd /tmp && export TMPDIR=/tmp && run stats_uniform 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_u -o uniform4k -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) || exit 1 ;;
    stats_zipf) (cd /tmp && export TMPDIR=/tmp && run stats_zipf 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_z -o zipf -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline) || exit 1 ;;
    pmc_uniform|pmc_zipf)
      cfg=${step#pmc_}; extra="--no-cpu-baseline"; [ $cfg = zipf ] && extra="--config zipf --no-buckets --no-cpu-baseline"
      (cd /tmp && export TMPDIR=/tmp &&
       run pmc_fetch_$cfg 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$cfg -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1 &&
       run pmc_write_$cfg 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$cfg -o pmc -- python3 $R/bench.py $extra --steps 5 --warmup 1) || exit 1
      if [ $cfg = zipf ]; then zipf_bytes; python3 tools/pmc_summary.py $O/pmc_fetch_zipf $O/pmc_write_zipf zipf $ZB bkd::crc_plan_chunks_kernel > $O/pmc_z.json || exit 1
      else python3 tools/pmc_summary.py $O/pmc_fetch_uniform $O/pmc_write_uniform uniform4k $((1048576*4100)) > $O/pmc_u.json || exit 1; fi ;;
    pmc_verify|pmc_package)  # the framed routes on their own: --digest-op verify | package
      op=${step#pmc_}; cfg=${op}4k
      # other kernels: the measured call's own launches (each bench also runs the other route once)
      if [ $op = verify ]; then mk=bkd::crc_verify_fused_kernel; ab=$((1048576*(4096+12+4)))
        ok=bkd::verify_gate_kernel,bkd::verify_header_kernel,bkd::plan_count_kernel,bkd::plan_scan_kernel,bkd::plan_emit_kernel,bkd::crc_plan_chunks_kernel,bkd::plan_combine_kernel,bkd::verify_finish_kernel
      else mk=bkd::crc_package_fused_kernel; ab=$((1048576*(4060+24+12+36+4))); ok=bkd::package_frame_kernel; fi
      (cd /tmp && export TMPDIR=/tmp &&
       run pmc_fetch_$cfg 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$cfg -o pmc -- python3 $R/bench.py --config verify4k --digest-op $op --steps 5 --warmup 1 &&
       run pmc_write_$cfg 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$cfg -o pmc -- python3 $R/bench.py --config verify4k --digest-op $op --steps 5 --warmup 1) || exit 1
      python3 tools/pmc_summary.py $O/pmc_fetch_$cfg $O/pmc_write_$cfg $cfg $ab $mk $ok > $O/pmc_$cfg.json || exit 1 ;;
    stats_verify|stats_package)
      op=${step#stats_}
      (cd /tmp && export TMPDIR=/tmp && run stats_$op 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$op -o $op -- python3 $R/bench.py --config verify4k --digest-op $op --steps 20 --warmup 5) || exit 1 ;;
    ab:*) run ab_$(date +%s%N) 900 python3 tools/ab_libs.py $(echo ${step#ab:} | tr , " ") ;;
    kstats:*) lib=${step#kstats:}; nm=$(basename $lib .so); (cd /tmp && export TMPDIR=/tmp && AB_ROUNDS=${AB_ROUNDS:-2} run kstats_$nm 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kstats_$nm -o k -- python3 $R/tools/ab_libs.py $R/$lib) || exit 1
      python3 tools/kstats.py $O/kstats_$nm > $O/kstats_$nm.txt && cat $O/kstats_$nm.txt ;;
    py:*) s=${step#py:}; run $(basename $s .py) 600 python3 $s ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
