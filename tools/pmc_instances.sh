#!/bin/bash
# PMC of the chunk kernel per library instance (identical copies of libbkdigest.so loaded side by
# side by tools/ab_libs.py): one rocprofv3 --pmc pass per counter set, rows grouped by Kernel_Id.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmci; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LIBS="$R/bookkeeper_amd/libbkdigest.so"
for i in 1 2 3 4 5; do cp $R/bookkeeper_amd/libbkdigest.so $O/lib_c$i.so; LIBS="$LIBS $O/lib_c$i.so"; done
i=0
for C in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY" \
         "TCC_TAG_STALL_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  AB_WORK=zipf AB_ROUNDS=3 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p -- python3 $R/tools/ab_libs.py $LIBS > $O/p$i.log 2>&1 || { echo "fail $i"; tail -5 $O/p$i.log; exit 1; }
  grep median $O/p$i.log
done
python3 - <<PY
import csv, glob, collections
for i in (1, 2, 3):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob("$O/p%d/**/*counter_collection.csv" % i, recursive=True):
        for r in csv.DictReader(open(path)):
            if "crc_plan_chunks_kernel" in r["Kernel_Name"]:
                vals[r["Kernel_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kid in sorted(vals, key=int):
        med = {k: sorted(v)[len(v) // 2] for k, v in vals[kid].items()}
        print("pass", i, "kernel", kid, " ".join("%s=%.4g" % (k, v) for k, v in sorted(med.items())))
PY
