#!/bin/bash
# r5: per-kernel times of the four-way pass (k_m4_rank, k_m4_merge) for each build in VARS
# (harness/bin/ab/liblabsort_<v>.so; "product" = the in-tree library), one rocprofv3 run each
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
export ALGO=merge
for v in ${VARS:-product}; do
  lib=""; [ "$v" != product ] && lib="$R/harness/bin/ab/liblabsort_$v.so"
  LABSORT_LIBRARY="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/rankab_$v" -o run -- python3 "$R/harness/exp/hist_time.py" > "$O/rankab_$v.log" 2>&1 || { tail -20 "$O/rankab_$v.log"; exit 1; }
  python3 - "$O/rankab_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "m4_" in r["Name"] or "merge_pass" in r["Name"] or "tile_sort" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0][-22:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
