#!/bin/bash
# Clock-adaptive fold: (1) parity tests of the one-entry-per-group paths with the fold4_main path
# forced (lib_b16 installed as the package library for the run), (2) same-process A/B of the
# adaptive default, the fixed compiler schedule (lib_noadapt) and the forced fold4_main (lib_b16),
# (3) the launch ramp with the shader clock for the three builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r03ad; mkdir -p $O; cd $R
cp bookkeeper_amd/libbkdigest.so /tmp/lib_default.so && cp tools/variants/lib_b16.so bookkeeper_amd/libbkdigest.so || exit 1
echo "== pytest with fold4_main forced"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_shard.py -k "uniform or indexed or package or golden or verify or lane or shard or config" > $O/pytest_b16.log 2>&1; rc=$?
cp /tmp/lib_default.so bookkeeper_amd/libbkdigest.so || exit 1
tail -2 $O/pytest_b16.log; [ $rc -eq 0 ] || exit $rc
W="uniform4k verify4k package4k indexed4k u8192_l8 u1024_l8 u512_l8"
echo "== ab order 1"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py bookkeeper_amd/libbkdigest.so tools/variants/lib_noadapt.so tools/variants/lib_b16.so > $O/ab1.log 2>&1 || { tail -20 $O/ab1.log; exit 1; }; grep median $O/ab1.log
echo "== ab order 2"
AB_ROUNDS=5 AB_WORK="$W" timeout -k 10 600 python3 tools/ab_libs.py tools/variants/lib_b16.so tools/variants/lib_noadapt.so bookkeeper_amd/libbkdigest.so > $O/ab2.log 2>&1 || { tail -20 $O/ab2.log; exit 1; }; grep median $O/ab2.log
echo "== ramp"
timeout -k 10 400 python3 tools/ramp_clock.py --rounds 4 --launches 60 bookkeeper_amd/libbkdigest.so tools/variants/lib_noadapt.so tools/variants/lib_b16.so > $O/ramp.log 2>&1 || { tail -5 $O/ramp.log; exit 1; }
python3 -c "
import json
for l in open('$O/ramp.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['lib'], d['round'], d['mean_5_25'], d['mean_50_end'])"
echo "== driver cmd"; timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || { tail -5 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log | cut -c1-200
echo done
