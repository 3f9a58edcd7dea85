#!/bin/bash
# Instruction mix and stall counters of the CRC kernels per tools/ab_libs.py workload (one
# rocprofv3 --pmc pass per counter set; AB_WORK names the workloads, the library is the in-tree one).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcw${PMC_TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
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
                for k in ("crc_plan_chunks_kernel", "crc_groups_kernel", "crc_stream_tiles_kernel"):
                    if k in r["Kernel_Name"]:
                        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            med[k][c] = sorted(v)[len(v) // 2]
    for k, m in med.items():
        print(w, k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(m.items())))
PY
