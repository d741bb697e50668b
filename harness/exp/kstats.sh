#!/bin/bash
# rocprofv3 kernel-trace stats of one python command; prints the labsort kernels' averages
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
D="$R/gpurun_out/kstats_${TAG:-x}"; rm -rf "$D"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- python3 "$@" > "$D.log" 2>&1 || { tail -5 "$D.log"; exit 1; }
python3 - "$D/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "labsort" in r["Name"]:
        print(f'  {r["Name"][:70]:70s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
