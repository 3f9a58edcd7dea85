#!/bin/bash
# SQ counters of the plan kernels (count / scan / emit / combine) and the chunk kernel on Zipf.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03o; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
B="SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
for set in A B; do
  ctr=${!set}
  echo "== pmc $set zipf"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${set}_zipf -o pmc -- python3 $R/bench.py --config zipf --no-buckets --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_${set}_zipf.log 2>&1 || { tail -5 $O/pmc_${set}_zipf.log; exit 1; }
done
cd $R && SQ_KERNELS="plan_count_kernel plan_scan_kernel plan_emit_kernel plan_combine_kernel crc_plan_chunks_kernel" python3 tools/sq_summary.py $O
