#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of bench.py for each
# library given (diagnostic builds); prints the labsort kernels' averages.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); D="$R/gpurun_out/ks_$i"; rm -rf "$D"
  echo "== $lib"
  LABSORT_LIBRARY="$R/$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-host-path --steps 10 --warmup 2 ${BENCH_ARGS:-} > "$D.log" 2>&1 || { tail -5 "$D.log"; exit 1; }
  python3 - "$D/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "labsort" in r["Name"]:
        print(f'  {r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
done
