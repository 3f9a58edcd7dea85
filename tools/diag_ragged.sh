#!/bin/bash
# rocprofv3 kernel trace of tools/diag_ragged.py and its per-workload kernel breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/diag_ragged -o diag -- python3 $R/tools/diag_ragged.py > $O/diag_ragged.log 2>&1 || { tail -30 $O/diag_ragged.log; exit 1; }
grep -v amdgpu.ids $O/diag_ragged.log
python3 $R/tools/diag_ragged.py --report $(ls $O/diag_ragged/*kernel_trace.csv $O/diag_ragged/*/*kernel_trace.csv 2>/dev/null | head -1) | tee $O/diag_ragged_report.txt
