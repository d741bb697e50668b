#!/bin/bash
# r6: four-way merge pass A/B -- the working tree's build (product) against harness/bin/ab
# builds named in VARS (default: base = HEAD before the change): merge tests, the randomized
# four-way stress check, alternating 2^28 merge sorts, and per-kernel rocprof times.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
TAG=${TAG:-m4ab}
VARS="${VARS:-base}"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sort.py -k "merge or four or pairs" > "$O/${TAG}_tests.log" 2>&1
tail -1 "$O/${TAG}_tests.log"
timeout -k 10 300 python3 -u tests/../harness/exp/m4_stress.py ${CASES:-300} > "$O/${TAG}_stress.log" 2>&1
tail -1 "$O/${TAG}_stress.log"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py \
  -k "merge and not pairs" > "$O/${TAG}_full.log" 2>&1
tail -1 "$O/${TAG}_full.log"
MODE=merge timeout -k 10 300 python3 -u harness/exp/pairs_ab.py radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so \
  $(for v in $VARS; do echo harness/bin/ab/liblabsort_$v.so; done) 4 > "$O/${TAG}_ab.log" 2>&1
cat "$O/${TAG}_ab.log"
if [ -n "${KV:-}" ]; then
  MODE=pairsmerge timeout -k 10 300 python3 -u harness/exp/pairs_ab.py radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so \
    $(for v in $VARS; do echo harness/bin/ab/liblabsort_$v.so; done) 3 > "$O/${TAG}_abkv.log" 2>&1
  cat "$O/${TAG}_abkv.log"
fi
cd /tmp && export TMPDIR=/tmp
export ALGO=merge
for v in product $VARS; do
  lib=""; [ "$v" != product ] && lib="$R/harness/bin/ab/liblabsort_$v.so"
  LABSORT_LIBRARY="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_$v" -o run -- \
    python3 "$R/harness/exp/hist_time.py" > "$O/${TAG}_$v.log" 2>&1
  python3 - "$O/${TAG}_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "m4_" in r["Name"] or "merge_pass" in r["Name"] or "tile_sort" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0][-24:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
