#!/bin/bash
# Lane-position finish (BKD_LANE_POS): GPU suite, same-process A/B against the lane-tree build in
# both library orders, SQ instruction counters per wave on 1- and 4-step heads and Zipf for both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03i; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
W="zipf zipf_crc32 zipf_heads_sorted chunk1s chunk4s mixed1k zipf_lt1k indexed4k uniform4k verify4k package4k u256_l4 u512_l8 u1024_l8"
echo "== ab order 1"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 500 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_tree.so > $O/ab1.log 2>&1 || { tail -5 $O/ab1.log; exit 1; }
grep median $O/ab1.log
echo "== ab order 2"; AB_ROUNDS=3 AB_WORK="$W" timeout -k 10 500 python3 tools/ab_libs.py tools/variants/lib_tree.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -5 $O/ab2.log; exit 1; }
grep median $O/ab2.log
cd /tmp; export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
cp -p $R/bookkeeper_amd/libbkdigest.so $O/lib_lanepos.so
for v in lanepos tree; do
  [ $v = tree ] && cp -p $R/tools/variants/lib_tree.so $R/bookkeeper_amd/libbkdigest.so
  for J in 1 4; do
    echo "== sq $v J=$J"
    HEADS_J=$J HEADS_MODES=2 timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $O/sq_$v/pmc_A_j$J -o pmc -- python3 $R/tools/diag_heads_j.py > $O/sq_${v}_j$J.log 2>&1 || { tail -5 $O/sq_${v}_j$J.log; cp -p $O/lib_lanepos.so $R/bookkeeper_amd/libbkdigest.so; exit 1; }
  done
  echo "== sq $v zipf"
  timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $O/sq_$v/pmc_A_zipf -o pmc -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline --steps 3 --warmup 1 > $O/sq_${v}_zipf.log 2>&1 || { tail -5 $O/sq_${v}_zipf.log; cp -p $O/lib_lanepos.so $R/bookkeeper_amd/libbkdigest.so; exit 1; }
done
cp -p $O/lib_lanepos.so $R/bookkeeper_amd/libbkdigest.so; rm -f $O/lib_lanepos.so
cd $R && python3 tools/sq_summary.py $O/sq_lanepos > $O/sq_lanepos.txt && python3 tools/sq_summary.py $O/sq_tree > $O/sq_tree.txt && cat $O/sq_lanepos.txt $O/sq_tree.txt | grep "per wave"
