#!/bin/bash
# Where the plan launches of config 3 spend their time: one rocprofv3 --pmc pass (SQ wave cycles,
# waits, VALU/LDS/SMEM issue) over a short Zipf bench, per plan kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03aj; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
timeout -k 10 -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/p1 -o p -- python3 $R/bench.py --config zipf --steps 3 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1 || { echo fail; tail -5 $O/p1.log; exit 1; }
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -k 10 -s KILL 150 rocprofv3 --pmc $C2 --output-format csv -d $O/p2 -o p -- python3 $R/bench.py --config zipf --steps 3 --warmup 1 --no-cpu-baseline > $O/p2.log 2>&1 || { echo fail2; tail -5 $O/p2.log; exit 1; }
python3 - <<PY
import csv, glob, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob("$O/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    med = {c: sorted(v)[len(v)//2] for c, v in d.items()}
    print(k, " ".join("%s=%.0f" % (c, v) for c, v in sorted(med.items())))
PY
echo done
