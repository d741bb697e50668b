#!/bin/bash
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
for lib in "$@"; do
  for p in 0 1; do
    LABSORT_TS_PERSIST=$p LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$lib.so" timeout -k 10 120 python3 "$R/harness/exp/ts_check.py" $p | sed "s/^/$lib /" || exit 1
  done
done
