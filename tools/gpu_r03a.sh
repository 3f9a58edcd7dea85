#!/bin/bash
# Round 3, first pass: the GPU suite (new: config-3 every entry vs the reference, two-rank config-4
# bench rehearsal), smoke, the clock-transient probes, and the host-route crossover.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03a; mkdir -p $O; cd $R
echo "== pytest gpu"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $O/pytest_gpu.log | tail -20; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "== ramp rounds (idle 2 s)"; timeout -k 10 120 python3 tools/ramp.py --rounds 3 --idle-ms 2000 > $O/ramp_rounds.log 2>&1 || { tail -5 $O/ramp_rounds.log; exit 1; }
echo "== ramp probe (plain nt read)"; timeout -k 10 120 ./tools/ramp_probe 200 2000 > $O/ramp_probe.log 2>&1 || { tail -5 $O/ramp_probe.log; exit 1; }
python3 - <<'PY'
import json, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/r03a"
for f in ("ramp_rounds.log", "ramp_probe.log"):
    for line in open(os.path.join(O, f)):
        if not line.startswith("{"):
            continue
        d = json.loads(line); ms = d["per_launch_ms"]
        print(f, d.get("round"), "by10:", [round(sum(ms[i:i+10]) / 10, 4) for i in range(0, len(ms), 10)])
PY
echo "== host route crossover"; timeout -k 10 600 python3 tools/host_route.py > $O/host_route.log 2>&1 || { tail -5 $O/host_route.log; exit 1; }
cat $O/host_route.log
