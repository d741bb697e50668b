#!/bin/bash
# pmc_sets.sh KRE TAG "SET1" "SET2" ... -- one rocprofv3 --pmc pass per counter set on the
# kernels matching KRE during `bench.py $BENCH_ARGS --steps 1 --warmup 1`; prints every
# dispatch's value per counter (gpurun_out/pmcs_TAG.txt)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
KRE="$1"; TAG="$2"; shift 2
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "$KRE" --output-format csv -d "$O/pmcs_${TAG}_$i" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$O/pmcs_${TAG}_$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$O/pmcs_${TAG}_$i.log"; exit 1; }
done
python3 - "$O" "$TAG" <<'PY' | tee "$O/pmcs_$2.txt"
import csv, sys, glob, collections
O, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{O}/pmcs_{tag}_*/run_counter_collection.csv")):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        by[r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    for k, v in sorted(by.items()):
        print(f"{k:28s}", " ".join(f"{x[1]/1e6:9.2f}M" for x in sorted(v)))
PY
