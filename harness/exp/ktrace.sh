#!/bin/bash
# ktrace.sh TAG LAST python-args... : kernel trace of one python command, last LAST kernels
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
T=$1; L=$2; shift 2
D="$R/gpurun_out/ktrace_$T"; rm -rf "$D"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$D" -o run -- python3 "$@" > "$D.log" 2>&1 || { tail -5 "$D.log"; exit 1; }
python3 "$R/harness/exp/ktrace.py" "$D/run_kernel_trace.csv" "$L"
