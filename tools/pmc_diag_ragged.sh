#!/bin/bash
# PMC of the chunk kernel per diag workload: one rocprofv3 --pmc pass per workload (kernel-trace off),
# counters: LDS busy / conflicts, VALU / LDS issue, wave cycles and waits, GPU busy cycles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcr; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for w in ${WL:-zipf_fullchunks_plan zipf_heads_plan zipf_lt1k_plan uniform4k_direct}; do
  DIAG_WORKLOADS=$w timeout -k 10 -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/$w -o p -- python3 $R/tools/diag_ragged.py > $O/$w.log 2>&1 || { echo "fail $w"; tail -5 $O/$w.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for w in "${WL:-zipf_fullchunks_plan zipf_heads_plan zipf_lt1k_plan uniform4k_direct}".split():
    vals = collections.defaultdict(list)
    for path in glob.glob("$O/%s/**/*counter_collection.csv" % w, recursive=True):
        for r in csv.DictReader(open(path)):
            if "crc_groups_kernel" in r["Kernel_Name"] or "crc_plan_chunks_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    med = {k: sorted(v)[len(v)//2] for k, v in vals.items()}
    g = med.get("GRBM_GUI_ACTIVE", 1)
    print(w, " ".join("%s=%.0f" % (k, v) for k, v in sorted(med.items())))
    print("   per GUI cycle: " + " ".join("%s=%.3f" % (k, v / g) for k, v in sorted(med.items()) if k != "GRBM_GUI_ACTIVE"))
PY
