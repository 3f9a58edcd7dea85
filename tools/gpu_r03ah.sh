#!/bin/bash
# Upper bound of the group finish's cost (measurement only): the launch ramp of the package build
# against one whose 8-lane finish is a plain XOR of the four streams (BKD_FINISH_PROBE=1, wrong
# digests, never shipped), with the shader clock probed after each launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ah; mkdir -p $O; cd $R
timeout -k 10 400 python3 tools/ramp_clock.py --no-check --probe --rounds 4 --launches 80 bookkeeper_amd/libbkdigest.so tools/variants/lib_nofinish.so > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
python3 -c "
import json
for l in open('$O/ramp.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'])"
echo done
