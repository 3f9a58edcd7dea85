#!/bin/bash
# BKD_FOLD_ASM=1 confirmation: the launch ramp (driver window) over five idle rounds, and a
# same-process A/B of the headline, verify and package routes in two library orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ac; mkdir -p $O; cd $R
echo "== ramp"
timeout -k 10 300 python3 tools/ramp_clock.py --rounds 5 --launches 60 bookkeeper_amd/libbkdigest.so tools/variants/lib_foldasm.so > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
python3 -c "
import json
for l in open('$O/ramp.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'])"
W="uniform4k verify4k package4k indexed4k"
echo "== ab order 1"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_foldasm.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_foldasm.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo done
