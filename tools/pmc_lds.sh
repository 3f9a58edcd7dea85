#!/bin/bash
# LDS issue stalls / bank conflicts of the chunk vs uniform kernel (one rocprofv3 --pmc pass per workload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcl${PMC_TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
for w in $AB_WORK; do
  AB_WORK=$w AB_ROUNDS=2 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$w -o p -- python3 $R/tools/ab_libs.py ${PMC_LIB:-$R/bookkeeper_amd/libbkdigest.so} > $O/$w.log 2>&1 || { echo "fail $w"; tail -5 $O/$w.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for w in "$AB_WORK".split():
    vals = collections.defaultdict(list)
    for path in glob.glob("$O/%s/**/*counter_collection.csv" % w, recursive=True):
        for r in csv.DictReader(open(path)):
            for k in ("crc_plan_chunks_kernel", "crc_groups_kernel"):
                if k in r["Kernel_Name"]:
                    vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(vals.items()):
        print(w, k, c, "%.4g" % sorted(v)[len(v) // 2])
PY
