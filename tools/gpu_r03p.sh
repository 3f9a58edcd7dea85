#!/bin/bash
# Round 3 (second session): GPU suite on the current tree, then the launch ramp with the shader
# clock beside it for the default build and the PF = 3 / 4 builds (tools/variants), then the
# driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03p; mkdir -p $O; cd $R
echo "== pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="bookkeeper_amd/libbkdigest.so tools/variants/pf/lib_pf3.so tools/variants/pf/lib_pf4.so"
echo "== ramp + clock"
timeout -k 10 300 python3 tools/ramp_clock.py --probe --rounds 2 $L > $O/ramp_clock.log 2>&1 || { tail -5 $O/ramp_clock.log; exit 1; }
python3 -c "
import json,sys
for l in open('$O/ramp_clock.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'], d['mhz'][:30])"
echo "== ramp, no probe"
timeout -k 10 300 python3 tools/ramp_clock.py --rounds 2 $L > $O/ramp_noprobe.log 2>&1 || { tail -5 $O/ramp_noprobe.log; exit 1; }
python3 -c "
import json,sys
for l in open('$O/ramp_noprobe.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'], d['per_launch_ms'][:30])"
echo "== ab short tail, order 1"
AB_ROUNDS=4 timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_noshort.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab short tail, order 2"
AB_ROUNDS=4 timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_noshort.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo "== zipf bench"
timeout -k 10 300 python3 bench.py --config zipf --steps 50 --warmup 20 > $O/zipf.log 2>&1 || { tail -5 $O/zipf.log; exit 1; }
tail -1 $O/zipf.log | cut -c1-600
echo "== driver cmd"
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.log 2>&1 || { tail -5 $O/driver.log; exit 1; }
tail -1 $O/driver.log | cut -c1-400
echo done
