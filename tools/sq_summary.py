"""Median per-dispatch SQ counters of the CRC kernels from rocprofv3 --pmc runs (tools/gpu_r03d.sh).

usage: sq_summary.py DIR  (DIR/pmc_<set>_<workload>/**/*counter_collection.csv)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = tuple(os.environ.get("SQ_KERNELS", "crc_plan_chunks_kernel crc_groups_kernel").split())


def main(d):
    res = defaultdict(dict)
    for path in glob.glob(os.path.join(d, "pmc_*_*", "**", "*counter_collection.csv"), recursive=True):
        work = os.path.relpath(path, d).split(os.sep)[0].split("_", 2)[2]
        for k in KERNELS:
            per = defaultdict(lambda: defaultdict(float))
            for row in csv.DictReader(open(path)):
                if k not in row["Kernel_Name"]:
                    continue
                per[row.get("Dispatch_Id", row.get("Correlation_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
            cols = defaultdict(list)
            for ctrs in per.values():
                for c, v in ctrs.items():
                    cols[c].append(v)
            key = work if len(KERNELS) == 1 or k in ("crc_plan_chunks_kernel", "crc_groups_kernel") else f"{work}:{k}"
            for c, v in cols.items():
                v.sort()
                res[key][c] = v[len(v) // 2]
    for work, ctr in sorted(res.items()):
        w = ctr.get("SQ_WAVES", 0) or 1
        print(work, json.dumps({k: round(v, 1) for k, v in sorted(ctr.items())}))
        print("   per wave:", {k: round(v / w, 1) for k, v in sorted(ctr.items()) if k != "SQ_WAVES"})
    json.dump(res, open(os.path.join(d, "sq_summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
