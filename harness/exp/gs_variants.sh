#!/bin/bash
# time the gathered radix of each variant library (harness/exp/libs) at 2^28, then
# per-kernel averages (rocprofv3) of each
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
for lib in "$@"; do
  LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$lib.so" timeout -k 10 120 python3 "$R/harness/exp/gs_check.py" time || exit 1
done
for lib in "$@"; do
  echo "== $lib"
  TAG=$lib LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$lib.so" bash "$R/harness/exp/kstats.sh" "$R/harness/exp/gs_check.py" prof | grep -v fill || exit 1
done
