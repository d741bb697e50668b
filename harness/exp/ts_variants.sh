#!/bin/bash
# merge sort / tile sort timing (harness/exp/ts_check.py) for each variant library
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
for lib in "$@"; do
  LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$lib.so" timeout -k 10 120 python3 "$R/harness/exp/ts_check.py" 0 | sed "s/^/$lib /" || exit 1
done
