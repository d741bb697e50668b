#!/bin/bash
# r5: onesweep rank loop with the lane-order check hoisted out of the per-key loop (hoist) vs HEAD,
# keys-only and key/value, alternating on one box.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
MODE=keys timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" harness/bin/ab/liblabsort_head.so harness/bin/ab/liblabsort_hoist.so 4 > "$O/hoist_keys.log" 2>&1 || { cat "$O/hoist_keys.log"; exit 1; }
cat "$O/hoist_keys.log"
MODE=pairs timeout -k 10 240 python -u "$R/harness/exp/pairs_ab.py" harness/bin/ab/liblabsort_r27.so harness/bin/ab/liblabsort_head.so harness/bin/ab/liblabsort_hoist.so 3 > "$O/hoist_pairs.log" 2>&1 || { cat "$O/hoist_pairs.log"; exit 1; }
cat "$O/hoist_pairs.log"
