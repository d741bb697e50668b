#!/bin/bash
# r5: four-way pass variants -- checks (product, 16 outputs per thread), merge-sort A/B against
# pairwise-only, per-kernel times of the product's four-way pass
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
VARS="${VARS:-m4k16}"
for lib in "" $(for v in $VARS; do echo "$R/harness/bin/ab/liblabsort_$v.so"; done); do
  LABSORT_LIBRARY="$lib" timeout -k 10 200 python -u "$R/harness/exp/m4_check.py" > "$O/m4c_check.log" 2>&1 || { cat "$O/m4c_check.log"; exit 1; }
  echo "check ${lib:-product}: $(grep -c ok "$O/m4c_check.log") ok, $(grep -c wrong "$O/m4c_check.log") wrong"
  grep wrong "$O/m4c_check.log" | head -3
done
MODE=merge timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/liblabsort.so $(for v in $VARS; do echo harness/bin/ab/liblabsort_$v.so; done) 3 > "$O/m4c_ab.log" 2>&1 || { cat "$O/m4c_ab.log"; exit 1; }
cat "$O/m4c_ab.log"
export ALGO=merge
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/m4c_prof" -o run -- python3 "$R/harness/exp/hist_time.py" > "$O/m4c_prof.log" 2>&1 || { tail -20 "$O/m4c_prof.log"; exit 1; }
cut -d, -f1-4 "$O"/m4c_prof/run_kernel_stats.csv | cut -c1-60,200-
