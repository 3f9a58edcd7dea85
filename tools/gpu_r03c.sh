#!/bin/bash
# Chunk-kernel cost by head step count J under rocprofv3 (kernel trace), and the counter list.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03c; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
HEADS_MODES=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_heads -o heads -- python3 $R/tools/diag_heads_j.py > $O/heads_prof.log 2>&1 || { tail -5 $O/heads_prof.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, os, json
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/r03c"
rows = []
for f in glob.glob(O + "/prof_heads/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# group: each J runs 13 crc_batch calls (3 warm + 10 timed) after its fill kernel
J = [int(x) for x in "1 2 3 4 6 8 12 16 24 32".split()]
seg, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "fill_splitmix64" in name:
        cur = {}
        seg.append(cur)
        continue
    if cur is None or "bkd::" not in name:
        continue
    cur.setdefault(name.split("<")[0], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for j, s in zip(J, seg):
    print(j, {k: round(sorted(v)[len(v) // 2], 2) for k, v in s.items()})
PY
