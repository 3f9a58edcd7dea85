#!/bin/bash
# PMC diagnosis: one rocprofv3 pass per counter group, uniform4k vs zipf; summary per kernel.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcdiag; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
for cfg in uniform4k zipf; do
  k=0
  for grp in "${GROUPS_[@]}"; do
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $O/${cfg}_$k -o p -- python3 $R/bench.py --config $cfg --no-buckets --steps 3 --warmup 1 --no-cpu-baseline > $O/${cfg}_$k.log 2>&1 || { echo "fail $cfg $k"; tail -5 $O/${cfg}_$k.log; exit 1; }
    k=$((k+1))
  done
done
python3 - <<PY
import csv, glob, collections
for cfg in ("uniform4k", "zipf"):
    vals = collections.defaultdict(list)
    for path in glob.glob("$O/%s_*/**/*counter_collection.csv" % cfg, recursive=True):
        for r in csv.DictReader(open(path)):
            if "crc_groups_kernel" in r["Kernel_Name"] or "crc_plan_chunks_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(cfg)
    for k2, v in sorted(vals.items()):
        v = sorted(v)
        print("   %-24s %16.0f  (n=%d)" % (k2, v[len(v)//2], len(v)))
PY
