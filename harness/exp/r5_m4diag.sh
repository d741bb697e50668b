#!/bin/bash
# r5: four-way merge pass timing builds (LABSORT_M4_DIAG 1/2/3: no level 1 / no level 2 / no co-rank
# searches) against the real one; merge-sort per-class launch times (outputs differ by design)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
MODE=merge timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so harness/bin/ab/liblabsort_m4d1.so harness/bin/ab/liblabsort_m4d2.so harness/bin/ab/liblabsort_m4d3.so 2 > "$O/m4diag.log" 2>&1 || { cat "$O/m4diag.log"; exit 1; }
cat "$O/m4diag.log"
bash "$R/harness/exp/r5_m4prof.sh"
python3 - "$O" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/pmc_m4_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        kn = "merge" if "k_m4_merge" in r["Kernel_Name"] else "rank" if "rank" in r["Kernel_Name"] else "other"
        acc[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kn, d in acc.items():
    print(kn, {k: round(sum(v) / len(v)) for k, v in sorted(d.items())})
PY
