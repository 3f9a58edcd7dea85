#!/bin/bash
# Head chunks vs uniform entries of the same step count J: the plan on unaligned heads, the plan on
# line-aligned whole-step heads, the uniform kernel on the same aligned entries; rocprofv3 kernel
# trace to split the chunk kernel from the plan kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03n; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
export HEADS_J="1 2 4 8 16 32"
HEADS_MODES="2" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_unal -o p -- python3 $R/tools/diag_heads_j.py > $O/unal.log 2>&1 || { tail -5 $O/unal.log; exit 1; }
HEADS_ALIGN=1 HEADS_MODES="2 3" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_al -o p -- python3 $R/tools/diag_heads_j.py > $O/al.log 2>&1 || { tail -5 $O/al.log; exit 1; }
grep -h '"J"' $O/unal.log $O/al.log
cd $R && python3 - <<'PY'
import csv, glob, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/r03n"
J = [int(x) for x in "1 2 4 8 16 32".split()]
for tag, modes in (("p_unal", ["plan"]), ("p_al", ["plan", "uniform"])):
    rows = []
    for f in glob.glob(O + f"/{tag}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "fill_splitmix64" in name:
            cur = {}
            segs.append(cur)
            continue
        if cur is None or "bkd::" not in name:
            continue
        cur.setdefault(name.split("<")[0].replace("bkd::", ""), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for j, s in zip(J, segs):
        print(tag, "J=%d" % j, {k: (len(v), round(sorted(v)[len(v) // 2], 2)) for k, v in s.items()})
PY
