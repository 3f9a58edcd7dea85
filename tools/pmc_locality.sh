#!/bin/bash
# Address-translation and L2 counters of the stream route's range kernel against the chunk kernel on
# the same workloads (tools/ab_libs.py; AB_MODE selects the route of the in-tree library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcl${PMC_TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for C in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
         "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for w in $AB_WORK; do
    AB_WORK=$w AB_ROUNDS=2 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i/$w -o p -- python3 $R/tools/ab_libs.py ${PMC_LIB:-$R/bookkeeper_amd/libbkdigest.so} > $O/p${i}_$w.log 2>&1 || { echo "fail $i $w"; tail -5 $O/p${i}_$w.log; exit 1; }
  done
done
python3 - <<PY
import csv, glob, collections
for w in "$AB_WORK".split():
    med = collections.defaultdict(dict)
    for i in (1, 2, 3):
        vals = collections.defaultdict(list)
        for path in glob.glob("$O/p%d/%s/**/*counter_collection.csv" % (i, w), recursive=True):
            for r in csv.DictReader(open(path)):
                for k in ("crc_plan_chunks_kernel", "crc_groups_kernel", "crc_stream_ranges_kernel"):
                    if k in r["Kernel_Name"]:
                        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            med[k][c] = sorted(v)[len(v) // 2]
    for k, m in med.items():
        print(w, k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(m.items())))
PY
