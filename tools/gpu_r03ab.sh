#!/bin/bash
# One fold step's 16 lookups issued together (BKD_FOLD_ASM=1, tools/variants/lib_foldasm.so):
# same-process A/B in two library orders (digests compared bit for bit), and the launch ramp with
# the shader clock for both builds (the driver's window, launches 5..24, is clock-limited).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/${RUN_TAG:-r03ab}; mkdir -p $O; cd $R
W="uniform4k indexed4k u8192_l8 u16384_l16 u1024_l8 u512_l8 zipf"
echo "== ab order 1"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_foldasm.so tools/variants/lib_foldasm2.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_foldasm2.so tools/variants/lib_foldasm.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo "== ramp"
timeout -k 10 300 python3 tools/ramp_clock.py --rounds 3 bookkeeper_amd/libbkdigest.so tools/variants/lib_foldasm.so tools/variants/lib_foldasm2.so > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
python3 -c "
import json
for l in open('$O/ramp.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'])"
echo done
