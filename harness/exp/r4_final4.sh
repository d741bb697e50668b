#!/bin/bash
# r4 (r28) validation after the merge pass's nontemporal loads: GPU suite, smoke, bench,
# committed profiles; then tile sort with nontemporal loads (MGX_TNT build) A/B.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
bash "$R/harness/exp/r4_final2.sh" || exit $?
cd "$R" || exit 1
for i in 1 2 3; do
  for L in base tnt; do
    ALGO=merge LABSORT_LIBRARY="$R/harness/exp/libs/liblabsort_$L.so" timeout -k 10 120 python "$R/harness/exp/hist_time.py" || exit 1
  done
done > "$R/gpurun_out/r4_tnt.txt" 2>&1
