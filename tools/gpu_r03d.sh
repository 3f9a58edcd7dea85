#!/bin/bash
# SQ counters of the chunk kernel on 1-step and 32-step chunks (tools/diag_heads_j.py) and on Zipf:
# instruction mix and where the waves wait. Two counter sets, one rocprofv3 pass each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03d; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY"
for set in A B; do
  ctr=${!set}
  for J in 1 32; do
    echo "== pmc $set J=$J"
    HEADS_J=$J HEADS_MODES=2 timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${set}_j$J -o pmc -- python3 $R/tools/diag_heads_j.py > $O/pmc_${set}_j$J.log 2>&1 || { tail -5 $O/pmc_${set}_j$J.log; exit 1; }
  done
  echo "== pmc $set zipf"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${set}_zipf -o pmc -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_${set}_zipf.log 2>&1 || { tail -5 $O/pmc_${set}_zipf.log; exit 1; }
  echo "== pmc $set uniform"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${set}_uni -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_${set}_uni.log 2>&1 || { tail -5 $O/pmc_${set}_uni.log; exit 1; }
done
cd $R && python3 tools/sq_summary.py $O
