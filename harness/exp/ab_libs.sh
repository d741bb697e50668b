#!/bin/bash
# ab_libs.sh ALGO LIB_A LIB_B [reps] -- alternating per-class launch times (hist_time.py) of
# two liblabsort builds (LABSORT_LIBRARY), 2^28 keys; each run has its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 ${4:-3}); do
  for L in "$2" "$3"; do
    ALGO=$1 LABSORT_LIBRARY="$R/$L" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done
